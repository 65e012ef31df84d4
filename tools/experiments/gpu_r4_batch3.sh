# GPU box: the sampler's sort-then-merge (bitwise test, then A/B at C2 / C3), the C1 bench with the
# size-ruled fused Adam, and the step tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/batch3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "merge or sampler" \
  > gpurun_out/batch3/t.txt 2>&1 || { tail -30 gpurun_out/batch3/t.txt; exit 1; }
tail -1 gpurun_out/batch3/t.txt
REP=2 bash tools/gpu_ab_env.sh "LONER_SAMPLER_MERGE=0|LONER_SAMPLER_MERGE=1" "--config C3;--config C2;--config C1" || exit 1
echo batch3 done
# the round's evidence with the defaults as committed (fused Adam by batch size)
bash tools/gpu_r4_all.sh "C2 C1 C4:--shard-of_8 C3 CAM" "" || exit 1
echo batch3 evidence done
