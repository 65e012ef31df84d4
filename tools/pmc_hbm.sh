# GPU box: FETCH_SIZE and WRITE_SIZE passes (one --pmc pass each, kernel trace only) over the bench
# command (the backward as the bench runs it: on-device rays, OGM-trained sampling) ->
# gpurun_out/pmc/FETCH_SIZE, gpurun_out/pmc/WRITE_SIZE (tools/refresh_profiles.py: per-launch bytes).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out}
CFG=${1:-C2}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmc/$c; mkdir -p $OUT/pmc/$c
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc/$c -o run -- \
    python3 $R/bench.py --config $CFG ${ARGS:-} --no-cpu-baseline --steps 20 > $OUT/pmc/$c/out.txt 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/pmc/$c/out.txt; exit 1; }
done
