# GPU box: the committed profile set for one config (tools/refresh_profiles.py turns it into profiles/):
#   bench.json (plain run, with cpu_baseline), prof/ (rocprofv3 --kernel-trace --stats of the same
#   bench command), pmc/FETCH_SIZE, pmc/WRITE_SIZE and pmc/MFMA (one --pmc pass each, kernel trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out}
CFG=${1:-C2}
cd $R
mkdir -p $OUT
timeout -k 10 300 python bench.py --config $CFG ${ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $OUT/prof $OUT/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $R/bench.py --config $CFG ${ARGS:-} --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err \
  || { tail -20 $OUT/bench_prof.err; exit 1; }
[ "${PMC:-1}" = 1 ] || { echo profiles done; exit 0; }  # PMC=0: the bench line and the kernel trace only
bash $R/tools/pmc_hbm.sh $CFG || exit 1
bash $R/tools/pmc_mfma.sh $CFG || exit 1
bash $R/tools/pmc_step.sh $CFG || exit 1
echo profiles done
