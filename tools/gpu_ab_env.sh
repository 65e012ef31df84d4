# GPU box: A/B of bench lines under environment settings.
# Usage: bash tools/gpu_ab_env.sh "<ENV=.. ENV2=..>|<ENV=..>" "<bench args>;<bench args>"  (the empty
# setting is allowed: "|LONER_X=1")
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/ab
mkdir -p $OUT
IFS='|' read -ra ENVS <<< "$1"
IFS=';' read -ra RUNS <<< "$2"
REP=${REP:-2}
for rep in $(seq $REP); do
for a in "${RUNS[@]}"; do
  for e in "${ENVS[@]}"; do
    env $e timeout -k 10 200 python bench.py $a --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python -c "
import json,sys; d=json.load(open('$OUT/b.json')); s=d['stage_ms']
print(f'[$e] [$a] {d[\"ms_per_step\"]:.4f} ms  ' + ' '.join(f'{k}={v:.4f}' for k,v in s.items()))"
  done
done
done
