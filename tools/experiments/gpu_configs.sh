# GPU box: bench lines (with CPU baselines) for C4, C3 and CAM, and a rocprofv3 --kernel-trace
# --stats summary of each config's bench command -> gpurun_out/cfg/<C>/{bench.json,prof/}.
set -o pipefail
R=$GRAFT_REPO_ROOT
for C in ${CONFIGS:-C4 C3 CAM}; do
  mkdir -p $R/gpurun_out/cfg/$C
  cd $R
  timeout -k 10 300 python bench.py --config $C > gpurun_out/cfg/$C/bench.json 2> gpurun_out/cfg/$C/bench.err || { tail -20 gpurun_out/cfg/$C/bench.err; exit 1; }
  cut -c1-200 gpurun_out/cfg/$C/bench.json
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/cfg/$C/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg/$C/prof -o run --output-format csv -- \
    python3 $R/bench.py --config $C --no-cpu-baseline > $R/gpurun_out/cfg/$C/bench_prof.json 2> $R/gpurun_out/cfg/$C/bench_prof.err \
    || { tail -20 $R/gpurun_out/cfg/$C/bench_prof.err; exit 1; }
done
echo configs done
