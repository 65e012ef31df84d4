# GPU box, round 3 committed profiles: per config, the bench line (with cpu_baseline) and the
# rocprofv3 --kernel-trace --stats summary of the same command; PMC passes (HBM bytes of the backward
# stage and of the whole step, MFMA busy) for the configs named in PMC.
#   bash tools/gpu_r3_profiles.sh "C2 C1 C4:--shard-of 8 C3 CAM C4"   (tools/refresh_profiles.py per config)
# Output under gpurun_out/${PROF_DIR:-r3p}/<config tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for spec in $1; do
  CFG=${spec%%:*}; ARGS=""; [ "$spec" != "$CFG" ] && ARGS="${spec#*:}"
  ARGS=${ARGS//_/ }
  TAG=$CFG$(echo "$ARGS" | tr -d ' -' | sed 's/shardof/s/')
  export OUT=$R/gpurun_out/${PROF_DIR:-r3p}/$TAG ARGS
  mkdir -p $OUT
  timeout -k 10 300 python bench.py --config $CFG $ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  echo "== $TAG"; cat $OUT/bench.json
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
      --output-format csv -- python3 $R/bench.py --config $CFG $ARGS --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err ) \
    || { tail -20 $OUT/bench_prof.err; exit 1; }
  if [[ " ${PMC:-} " == *" $TAG "* ]]; then
    bash $R/tools/pmc_hbm.sh $CFG || exit 1
    bash $R/tools/pmc_mfma.sh $CFG || exit 1
    bash $R/tools/pmc_step.sh $CFG || exit 1
  fi
done
echo profiles done
