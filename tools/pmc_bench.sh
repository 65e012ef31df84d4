# PMC passes over the bench command (GPU box): one rocprofv3 --pmc pass per counter group, kernel
# trace only, each under its own time limit.  Output: gpurun_out/pmcb/<pass>/...; summary by
# tools/pmc_summary.py gpurun_out/pmcb.   Usage: bash tools/pmc_bench.sh [lib.so]
set -o pipefail
R=$GRAFT_REPO_ROOT
LIB=${1:-$R/loner_amd/_lib/libloner_amd.so}
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  D=${OUT:-$R/gpurun_out}/pmcb
  mkdir -p $D/$tag
  LONER_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
    -d $D/$tag -o run -- python3 $R/bench.py ${ARGS:-} --no-cpu-baseline --steps 10 > $D/$tag/out.txt 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run sqA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES
run sqB SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM
run sqC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT
python3 $R/tools/pmc_summary.py ${OUT:-$R/gpurun_out}/pmcb | tee ${OUT:-$R/gpurun_out}/pmcb/summary.txt | grep -A1 -E "k_bwd_scatter_rows|k_bwd_accum|k_hashgrid_fwd|k_mlp_bwd|k_field_wave|k_sigma_fwd|k_composite"
