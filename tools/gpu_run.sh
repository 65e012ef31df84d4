# GPU box: the one parameterised measurement script (round 5 on; the round-specific batch scripts of
# earlier rounds are in git history, listed in tools/README.md).  Parts run in the order given; each
# GPU step has its own time limit and the script stops at the first failure.
#   bash tools/gpu_run.sh <tag> <part> [<part> ...]
# parts:
#   suite                  the whole -m gpu suite (-> suite.log)
#   tests:<file[,file]>    some GPU test files
#   bench:<spec>           one bench line, no cpu_baseline (spec: C2, C1, C4_--shard-of_8, ...)
#   prof:<spec>            the committed profile set of one config (bench line with cpu_baseline +
#                          rocprofv3 kernel stats, tools/gpu_r3_profiles.sh)
#   pipeline               tools/exp_pipeline.py C2 (row-pipelined step feasibility)
#   pmccam                 PMC passes over the CAM bench (tools/pmc_cam.sh)
#   slack:<spec>           kernel trace of one config + tools/join_slack.py
#   ab:<envs>:<runs>       tools/gpu_ab_env.sh A/B (envs "A=1|A=0", runs "--config C2;--config C1", '_' = ' ')
#   py:<script+args>       any python tool (+ = space)
# Output: gpurun_out/<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
spec_args() {  # C4_--shard-of_8 -> CFG=C4 ARGS="--shard-of 8" STAG=C4s8
  CFG=${1%%_*}; ARGS=""; [ "$1" != "$CFG" ] && ARGS="${1#*_}"; ARGS=${ARGS//_/ }
  STAG=$CFG$(echo "$ARGS" | tr -d ' -' | sed 's/shardof/s/')
}
for part in "$@"; do
  kind=${part%%:*}; arg=${part#*:}
  echo "== $part"
  case $kind in
    suite)
      timeout -k 10 900 python -u -m pytest -v -x --timeout 120 --timeout-method thread -m gpu tests \
        > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
      tail -1 $O/suite.log ;;
    tests)
      timeout -k 10 600 python -u -m pytest -v -x --timeout 120 --timeout-method thread -m gpu ${arg//,/ } \
        > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
      tail -1 $O/tests.log ;;
    bench)
      spec_args $arg
      timeout -k 10 300 python bench.py --config $CFG $ARGS --no-cpu-baseline > $O/bench_$STAG.json 2> $O/bench_$STAG.err \
        || { tail -20 $O/bench_$STAG.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/bench_$STAG.json').read().strip().splitlines()[-1]); s=d.get('stage_ms', {})
print('$STAG', round(d['ms_per_step'], 4), ' '.join(f'{k}={v:.4f}' for k, v in s.items()))" ;;
    prof)
      spec_args $arg
      PROF_DIR=$TAG bash tools/gpu_r3_profiles.sh "${CFG}${ARGS:+:${ARGS// /_}}" || exit 1 ;;
    pipeline)
      timeout -k 10 300 python -u tools/exp_pipeline.py C2 ${arg#pipeline} > $O/pipeline.txt 2>&1 || { tail -20 $O/pipeline.txt; exit 1; }
      cat $O/pipeline.txt ;;
    pmccam)
      bash tools/pmc_cam.sh > $O/pmccam.txt 2>&1 || { tail -20 $O/pmccam.txt; exit 1; }
      cp -r $R/gpurun_out/pmccam $O/ 2>/dev/null; tail -5 $O/pmccam.txt ;;
    slack)
      spec_args $arg
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $O/trace_$STAG -o run -- python3 $R/bench.py --config $CFG $ARGS --no-cpu-baseline \
          > $O/trace_$STAG.json 2> $O/trace_$STAG.err ) || { tail -20 $O/trace_$STAG.err; exit 1; }
      f=$(find $O/trace_$STAG -name "*kernel_trace.csv" | head -1)
      python3 tools/join_slack.py $f | tee $O/slack_$STAG.json ;;
    ab)
      envs=${arg%%:*}; runs=${arg#*:}
      REP=${REP:-2} bash tools/gpu_ab_env.sh "$envs" "${runs//_/ }" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
      cat $O/ab.txt ;;
    py)
      timeout -k 10 400 python -u ${arg//+/ } > $O/py.txt 2>&1 || { tail -20 $O/py.txt; exit 1; }
      tail -30 $O/py.txt ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
echo "$TAG done"
