# GPU box: texture-unit / cache-request PMC pass over tools/exp_kernels.py -> gpurun_out/pmc/units
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export EXP_STEPS=${EXP_STEPS:-5}
rm -rf $R/gpurun_out/pmc/units; mkdir -p $R/gpurun_out/pmc/units
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TD_BUSY_avr TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $R/gpurun_out/pmc/units -o run -- python3 $R/tools/exp_kernels.py \
  > $R/gpurun_out/pmc/units/out.txt 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc/units/out.txt; exit 1; }
