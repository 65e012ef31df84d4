# GPU box: the committed profile set for one config (tools/refresh_profiles.py turns it into profiles/):
#   bench.json (plain run, with cpu_baseline), prof/ (rocprofv3 --kernel-trace --stats of the same
#   bench command), pmc/FETCH_SIZE, pmc/WRITE_SIZE and pmc/MFMA (one --pmc pass each, kernel trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT
CFG=${1:-C2}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config $CFG > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof $R/gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- \
  python3 $R/bench.py --config $CFG --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err \
  || { tail -20 $R/gpurun_out/bench_prof.err; exit 1; }
bash $R/tools/pmc_hbm.sh $CFG || exit 1
bash $R/tools/pmc_mfma.sh $CFG || exit 1
bash $R/tools/pmc_step.sh $CFG || exit 1
echo profiles done
