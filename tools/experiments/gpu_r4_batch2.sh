# GPU box: the fused Adam's bitwise test and A/B (eight parameters per thread), the composite kernel at
# four waves per SIMD.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/batch2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rays.py -k "fused or graph" \
  > gpurun_out/batch2/t.txt 2>&1 || { tail -30 gpurun_out/batch2/t.txt; exit 1; }
tail -1 gpurun_out/batch2/t.txt
bash tools/gpu_r4_fused.sh || exit 1
bash tools/gpu_ab_libs.sh "cw4" || exit 1
echo batch2 done
# the round's evidence with the defaults as committed: the whole suite, the profile set, PMC at C2
PMC="C2" bash tools/gpu_r4_all.sh "C2 C1 C4:--shard-of_8 C3 CAM" "" || exit 1
echo batch2 evidence done
