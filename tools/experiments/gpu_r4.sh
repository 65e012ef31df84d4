# GPU box, round 4 measurements: graph-replay tests and benches (C1, C2, C4 shard 1/8, each with and
# without the HIP graph), the FETCH_SIZE / WRITE_SIZE calibration microbenchmark, the backward's PMC
# split (eager path), and the side-stream join slack at shard 1/8 from a kernel trace.
#   bash tools/gpu_r4.sh [parts]      parts: any of "tests bench calib pmc slack" (default: all)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
PARTS=${1:-"tests bench graphcost calib pmc slack"}
cd $R
if [[ " $PARTS " == *" tests "* ]]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rays.py tests/test_gpu_parity.py \
    tests/test_gpu_dist.py tests/test_gpu_step.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
  tail -2 $O/tests.txt
fi
if [[ " $PARTS " == *" bench "* ]]; then
  for spec in C1 C2 C4:--shard-of_8; do
    CFG=${spec%%:*}; ARGS=""; [ "$spec" != "$CFG" ] && ARGS="${spec#*:}"; ARGS=${ARGS//_/ }
    TAG=$CFG$(echo "$ARGS" | tr -d ' -' | sed 's/shardof/s/')
    for g in 1 0; do
      LONER_GRAPH=$g timeout -k 10 200 python bench.py --config $CFG $ARGS --no-cpu-baseline > $O/bench_${TAG}_g$g.json \
        2> $O/bench_${TAG}_g$g.err || { tail -20 $O/bench_${TAG}_g$g.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$O/bench_${TAG}_g$g.json').read().strip().splitlines()[-1]); print('$TAG graph=$g', d['ms_per_step'], d['value'])"
    done
  done
fi
if [[ " $PARTS " == *" graphcost "* ]]; then
  for c in C1 C2; do timeout -k 10 120 python tools/graph_cost.py $c | tee $O/graph_cost_$c.json || exit 1; done
fi
if [[ " $PARTS " == *" calib "* ]]; then
  hipcc -O3 --offload-arch=gfx950 tools/ubench/ubench_fetch.hip -o /tmp/ubf || exit 1
  ( cd /tmp && export TMPDIR=/tmp
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/calib_$c -o run -- /tmp/ubf \
        > $O/calib_$c.out 2>&1 || { tail -5 $O/calib_$c.out; exit 1; }
    done ) || exit 1
  python3 tools/pmc_summary.py $O/calib_FETCH_SIZE > $O/calib_fetch.txt && python3 tools/pmc_summary.py $O/calib_WRITE_SIZE > $O/calib_write.txt
  cat $O/calib_fetch.txt $O/calib_write.txt
  grep kr16 $O/calib_FETCH_SIZE.out | tail -1; tail -1 $O/calib_FETCH_SIZE.out
fi
if [[ " $PARTS " == *" pmc "* ]]; then
  LONER_GRAPH=0 bash tools/pmc_bench.sh > $O/pmc_split.txt 2>&1 || { tail -20 $O/pmc_split.txt; exit 1; }
  tail -20 $O/pmc_split.txt
fi
if [[ " $PARTS " == *" slack "* ]]; then
  for g in 0; do
    ( cd /tmp && export TMPDIR=/tmp && LONER_GRAPH=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $O/trace_C4s8_g$g -o run -- python3 $R/bench.py --config C4 --shard-of 8 --no-cpu-baseline \
        > $O/trace_C4s8_g$g.json 2> $O/trace_C4s8_g$g.err ) || { tail -20 $O/trace_C4s8_g$g.err; exit 1; }
    f=$(find $O/trace_C4s8_g$g -name "*kernel_trace.csv" | head -1)
    python3 tools/join_slack.py $f | tee $O/slack_C4s8_g$g.json
  done
fi
echo r4 done
