# GPU box: A/B of an environment switch on the default library: bench stage times per setting (REP rounds,
# interleaved).   bash tools/gpu_ab_env.sh VAR "v1 v2 ..." ["<bench args>"]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/abenv
mkdir -p $OUT
REP=${REP:-2}
for rep in $(seq $REP); do
  for v in $2; do
    env $1=$v timeout -k 10 200 python bench.py ${3:-} --no-cpu-baseline > $OUT/b_$v.json 2> $OUT/b_$v.err \
      || { tail -20 $OUT/b_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]); s=d['stage_ms']
print(f'[$1=$v] {d[\"ms_per_step\"]:.4f} ms  ' + ' '.join(f'{k}={v:.4f}' for k,v in s.items()), flush=True)"
  done
done
echo abenv done
