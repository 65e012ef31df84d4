# PMC passes over tools/exp_kernels.py (GPU box): one rocprofv3 --pmc pass per counter group,
# kernel-trace only.  Output: gpurun_out/pmc/<pass>/...   Usage: bash tools/pmc.sh [lib.so]
set -o pipefail
R=$GRAFT_REPO_ROOT
LIB=${1:-$R/loner_amd/_lib/libloner_amd.so}
cd /tmp && export TMPDIR=/tmp
export EXP_STEPS=${EXP_STEPS:-5}
run() {
  tag=$1; shift
  mkdir -p $R/gpurun_out/pmc/$tag
  LONER_AMD_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
    -d $R/gpurun_out/pmc/$tag -o run -- python3 $R/tools/exp_kernels.py > $R/gpurun_out/pmc/$tag/out.txt 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run sqA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES
run sqB SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM
run fetch FETCH_SIZE
run write WRITE_SIZE
