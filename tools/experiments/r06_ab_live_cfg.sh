# LONER_LIVE_BWD=0 / 1 / auto on one bench config (trained field): bash tools/experiments/r06_ab_live_cfg.sh "--config C4 --shard-of 8"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06f
for v in 0 1 auto 0 1; do
  LONER_LIVE_BWD=$v timeout -k 10 200 python bench.py $1 --no-cpu-baseline --steps 40 > gpurun_out/r06f/l.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r06f/l.json').read().strip().splitlines()[-1])
print('live=$v', round(d['ms_per_step'],4), 'bwd', round(d['stage_ms']['grid_bwd'],4), 'dead', round(d['dsigma_zero_frac'],3), 'dead waves', round(d['dead_wave_frac'],3), d['backward_stage']['backward'][:4])"
done
