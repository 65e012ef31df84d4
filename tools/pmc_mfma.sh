# GPU box: one --pmc pass (kernel trace only) of MFMA busy cycles and GPU-active cycles over the bench
# command -> gpurun_out/pmc/MFMA (tools/refresh_profiles.py reads it).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out}
cd /tmp && export TMPDIR=/tmp
CFG=${1:-C2}
rm -rf $OUT/pmc/MFMA; mkdir -p $OUT/pmc/MFMA
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d $OUT/pmc/MFMA -o run -- python3 $R/bench.py --config $CFG ${ARGS:-} --no-cpu-baseline --steps 20 > $OUT/pmc/MFMA/out.txt 2>&1
rc=$?; echo "pmc MFMA rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/pmc/MFMA/out.txt; exit 1; }
