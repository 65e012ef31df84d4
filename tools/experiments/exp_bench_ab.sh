# GPU box: the bench (default config unless BENCH_ARGS) under rocprofv3 --kernel-trace --stats for the
# default library and every variant under loner_amd/_lib/variants/, then the named kernels' average
# time and the bench's ms/step per variant.  Usage: bash tools/experiments/exp_bench_ab.sh k_bwd_accum ...
set -o pipefail
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/bab
cd /tmp && export TMPDIR=/tmp
shopt -s nullglob
for lib in $R/loner_amd/_lib/libloner_amd.so $R/loner_amd/_lib/variants/*.so; do
  tag=$(basename $lib .so)
  O=$R/gpurun_out/bab/$tag
  mkdir -p $O
  LONER_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "FAIL $tag"; tail -20 $O/bench.err; exit 1; }
  F=$(find $O -name '*kernel_stats.csv' | head -1)
  echo "== $tag: $(python3 -c "import json;print(round(json.load(open('$O/bench.json'))['ms_per_step'],4))") ms/step"
  python3 - "$F" "$@" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for k in sys.argv[2:]:
    for r in rows:
        if k + "(" in r["Name"] or k + "<" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
