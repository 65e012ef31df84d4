# GPU box: the fused table Adam (LONER_FUSED_ADAM) against the separate Adam: bench A/B at C2 and C1,
# then the training digest under each (bitwise the same parameters and moments expected).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/fused
REP=2 bash tools/gpu_ab_env.sh "LONER_FUSED_ADAM=1|LONER_FUSED_ADAM=0" "--config C2;--config C1" || exit 1
for f in 1 0; do
  LONER_FUSED_ADAM=$f timeout -k 10 120 python tools/lib_digest.py 3 > gpurun_out/fused/d_$f.txt 2>&1 || { tail -20 gpurun_out/fused/d_$f.txt; exit 1; }
  echo "fused=$f $(tail -1 gpurun_out/fused/d_$f.txt)"
done
