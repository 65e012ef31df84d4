# A/B of the live backward (LONER_LIVE_BWD=0 / 1) in both regimes of bench.py --field trained, then other configs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06e
for v in 0 1; do
  LONER_LIVE_BWD=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/r06e/live$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r06e/live$v.json').read().strip().splitlines()[-1]); f=d['from_init']
print('live=$v trained', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['stage_ms'].items()})
print('live=$v init   ', round(f['ms_per_step'],4), {k: round(x,4) for k,x in f['stage_ms'].items()})"
done
