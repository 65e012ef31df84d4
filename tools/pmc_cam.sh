# PMC passes over the CAM bench (GPU box), kernel-trace only.  Output (PMC_CONFIG, default CAM): gpurun_out/pmccam/<pass>/...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  mkdir -p $R/gpurun_out/pmccam/$tag
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
    -d $R/gpurun_out/pmccam/$tag -o run -- python3 $R/bench.py --config ${PMC_CONFIG:-CAM} --steps 3 --warmup 1 --no-cpu-baseline \
    > $R/gpurun_out/pmccam/$tag/out.txt 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run sqA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES
run sqB SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA
run mf SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
