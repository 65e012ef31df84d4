# GPU box: given pytest selection (default: the gpu suite) then the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/q
SEL=${1:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1 || { tail -60 gpurun_out/q/pytest.log; exit 1; }
tail -3 gpurun_out/q/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { tail -20 gpurun_out/q/bench.err; exit 1; }
cat gpurun_out/q/bench.json
