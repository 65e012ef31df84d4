# GPU box: tools/experiments/exp_variants.sh, then the average time of the named kernels per variant.
# Usage: bash tools/experiments/exp_ab_run.sh k_bwd_accum k_bwd_scatter_rows ...
set -o pipefail
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/exp
bash $R/tools/experiments/exp_variants.sh || exit 1
for d in $R/gpurun_out/exp/*/; do
  F=$(find $d -name '*kernel_stats.csv' | head -1)
  echo "== $(basename $d)"
  python3 - "$F" "$@" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for k in sys.argv[2:]:
    for r in rows:
        if k + "(" in r["Name"] or k + "<" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
