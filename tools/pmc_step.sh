# GPU box: FETCH_SIZE and WRITE_SIZE passes (one --pmc pass each, kernel trace only) over the bench
# command itself (every kernel of the step) -> gpurun_out/pmc_step/{FETCH_SIZE,WRITE_SIZE};
# tools/refresh_profiles.py turns them into profiles/<tag>_traffic_<cfg>_step.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out}
CFG=${1:-C2}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmc_step/$c; mkdir -p $OUT/pmc_step/$c
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_step/$c -o run -- \
    python3 $R/bench.py --config $CFG ${ARGS:-} --no-cpu-baseline --steps 20 > $OUT/pmc_step/$c/out.txt 2>&1
  rc=$?; echo "pmc_step $c rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/pmc_step/$c/out.txt; exit 1; }
done
