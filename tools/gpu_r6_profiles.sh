# GPU box, round 6 profile set of one optimiser-step config on the TRAINED field (bench.py --field trained):
#   1. the bench line (with cpu_baseline: from-init steps, the untimed pre-training, the trained window), which
#      also saves the pre-trained field to /tmp (--field-cache);
#   2. rocprofv3 --kernel-trace --stats of the same command loading that field (no from-init steps, no
#      pre-training: the kernel statistics are the trained window's steps only);
#   3. (PMC=1) the PMC passes over the same command: HBM bytes of the backward stage and of the whole step,
#      MFMA busy, L2 requests + texture-addresser busy, SQ counters (LDS bank conflicts, VALU / LDS activity).
#   bash tools/gpu_r6_profiles.sh C2 [tag]          (tools/refresh_profiles.py <round> C2 gpurun_out/<tag>/C2)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
CFG=${1:-C2}
TAG=${2:-r6p}
FC=/tmp/loner_field_$CFG.pt
export OUT=$R/gpurun_out/$TAG/$CFG ARGS="--field-cache $FC ${EXTRA:-}"
mkdir -p $OUT
rm -f $FC
timeout -k 10 400 python bench.py --config $CFG $ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo "== $CFG"; python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['stage_ms'])"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
    --output-format csv -- python3 $R/bench.py --config $CFG $ARGS --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err ) \
  || { tail -20 $OUT/bench_prof.err; exit 1; }
if [ "${PMC:-0}" = 1 ]; then
  bash $R/tools/pmc_hbm.sh $CFG || exit 1
  bash $R/tools/pmc_mfma.sh $CFG || exit 1
  bash $R/tools/pmc_step.sh $CFG || exit 1
  bash $R/tools/pmc_l2req.sh $CFG || exit 1
  [ "$CFG" = C2 ] && { bash $R/tools/pmc_bench.sh || exit 1; }
fi
echo profiles done
