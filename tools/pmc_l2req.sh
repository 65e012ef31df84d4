# GPU box: L2 request counters over the bench command (one --pmc pass per group, kernel trace only):
# how many cache lines each kernel asks the L2 for (TCP_TCC_READ_REQ: vector-L1 misses sent to the L2)
# and how many of them hit.  The encode is priced against the L2 request rate in DESIGN.md section 4
# (tools/ubench/ubench_gather.hip: ~270 G lines/s for an L2-resident table).
# Output: gpurun_out/pmcl2/<pass>/..., summary by tools/pmc_summary.py gpurun_out/pmcl2.
# Usage: bash tools/pmc_l2req.sh [config]
set -o pipefail
R=$GRAFT_REPO_ROOT
CFG=${1:-C2}
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  D=${OUT:-$R/gpurun_out}/pmcl2${TAG:-}
  mkdir -p $D/$tag
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
    -d $D/$tag -o run -- python3 $R/bench.py --config $CFG ${ARGS:-} --no-cpu-baseline --steps 10 \
    > $D/$tag/out.txt 2>&1
  rc=$?
  echo "pmc $tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run l2a TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum
run l2b TCC_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE
D=${OUT:-$R/gpurun_out}/pmcl2${TAG:-}
python3 $R/tools/pmc_summary.py $D > $D/summary.txt
grep -A1 -E "k_hashgrid_fwd|k_bwd_scatter_rows|k_bwd_accum|k_mlp_bwd|k_sigma_fwd" $D/summary.txt
