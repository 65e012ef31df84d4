# GPU box: timing only (no tests) of the default build and every variant (tools/experiments/exp_variants.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/exp
bash tools/experiments/exp_variants.sh
