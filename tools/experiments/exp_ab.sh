# GPU box: A/B of an environment switch of tools/exp_kernels.py under rocprofv3 --stats.
#   bash tools/experiments/exp_ab.sh VAR   -> gpurun_out/exp/VAR0, gpurun_out/exp/VAR1
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  mkdir -p $R/gpurun_out/exp/$1$v
  env $1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exp/$1$v -o run --output-format csv -- \
    python3 $R/tools/exp_kernels.py > $R/gpurun_out/exp/$1$v/out.txt 2>&1 || { tail -20 $R/gpurun_out/exp/$1$v/out.txt; exit 1; }
  echo "$1=$v: $(grep ms/step $R/gpurun_out/exp/$1$v/out.txt)"
done
