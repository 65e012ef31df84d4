# GPU box: backward-relevant parity tests (plus any extra pytest args), then the A/B timing of the
# default build against every variant library (tools/experiments/exp_variants.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step.py tests/test_gpu_fullsize.py tests/test_gpu_compat.py "$@" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t/pytest.log 2>&1 || { tail -40 gpurun_out/t/pytest.log; exit 1; }
tail -2 gpurun_out/t/pytest.log
rm -rf gpurun_out/exp
bash tools/experiments/exp_variants.sh
