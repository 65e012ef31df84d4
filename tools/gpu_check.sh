set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv rocpd -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
cat $R/gpurun_out/bench_prof.json
find $R/gpurun_out/prof -name '*stats*'
