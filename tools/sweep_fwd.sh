# encode launch-shape sweep (GPU box): bash tools/sweep_fwd.sh "<env>;<env>;..."
set -o pipefail
cd $GRAFT_REPO_ROOT
IFS=';' read -ra RUNS <<< "${1:-}"
for cfg in "${RUNS[@]}"; do
  echo "== $cfg"
  env $cfg ALONE_ONLY=1 timeout -k 10 120 python tools/exp_overlap.py ${CONFIG:-C2} 2>&1 | grep alone || exit 1
done
