# GPU box: 2-rank rehearsal of bench.py's data-parallel path on one GPU (gloo), then N=1 for reference.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/dist
LONER_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/dist/bench2.json 2> gpurun_out/dist/bench2.err || { tail -30 gpurun_out/dist/bench2.err; exit 1; }
cat gpurun_out/dist/bench2.json
