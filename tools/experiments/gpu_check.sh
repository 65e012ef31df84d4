# GPU box: parity suite, bench, rocprof kernel stats of the bench (round-1 refresh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/chk
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1 || { tail -40 gpurun_out/chk/pytest.log; exit 1; }
tail -3 gpurun_out/chk/pytest.log
timeout -k 10 300 python bench.py > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err || { tail -20 gpurun_out/chk/bench.err; exit 1; }
cat gpurun_out/chk/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/chk/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/chk/bench_prof.json 2>&1 || { tail -20 $R/gpurun_out/chk/bench_prof.json; exit 1; }
tail -1 $R/gpurun_out/chk/bench_prof.json
