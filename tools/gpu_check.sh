# Round refresh on the GPU box: GPU tests, the default bench line, a rocprofv3 --stats profile of the
# same bench command, and PMC FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel-trace only).
# Output under gpurun_out/; tools/refresh_profiles.py turns it into profiles/ files.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof gpurun_out/pmc
CFG=${CFG:-C2}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --config $CFG > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- $BENCH \
  > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $R/gpurun_out/pmc/$C
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$C -o run -- \
    python3 $R/bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/pmc/$C/out.txt 2>&1 \
    || { echo "PMC_FAIL $C"; tail -20 $R/gpurun_out/pmc/$C/out.txt; exit 1; }
done
echo DONE
