# GPU box: MALL write->read micro-benchmark, then the gpu suite and the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r2a
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/r2a/ubench_mall tools/ubench/ubench_mall.hip 2> /dev/null || exit 1
timeout -k 10 120 gpurun_out/r2a/ubench_mall > gpurun_out/r2a/mall.txt 2>&1 || exit 1
cat gpurun_out/r2a/mall.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 || { tail -40 gpurun_out/r2a/pytest.log; exit 1; }
tail -3 gpurun_out/r2a/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || { tail -20 gpurun_out/r2a/bench.err; exit 1; }
cat gpurun_out/r2a/bench.json
