# GPU box, round 4 batch: the fused-Adam bitwise test and A/B, the colour-grid group size on CAM, the
# scatter level-order variants, and the encode's L2 / TA counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/batch
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rays.py \
  > gpurun_out/batch/rays_tests.txt 2>&1 || { tail -30 gpurun_out/batch/rays_tests.txt; exit 1; }
tail -1 gpurun_out/batch/rays_tests.txt
bash tools/gpu_r4_fused.sh || exit 1
REP=2 bash tools/gpu_ab_libs.sh "col1" "--config CAM" || exit 1
bash tools/gpu_ab_libs.sh "rotall rot32" || exit 1
bash tools/pmc_l2req.sh C2 > gpurun_out/batch/l2req.txt 2>&1 || { tail -5 gpurun_out/batch/l2req.txt; exit 1; }
tail -12 gpurun_out/batch/l2req.txt
echo batch done
