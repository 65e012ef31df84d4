# GPU box, round 3: gpu suite (optional), then bench lines and kernel-stats profiles for the given
# configs.  Usage: bash tools/gpu_r3.sh [tests|notests] "<bench args>;<bench args>;..."
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r3
mkdir -p $OUT
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
IFS=';' read -ra RUNS <<< "${2:-}"
i=0
for a in "${RUNS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$i.json 2> $OUT/bench_$i.err \
    || { tail -20 $OUT/bench_$i.err; exit 1; }
  echo "== $a"; cat $OUT/bench_$i.json
  if [ -n "${PROF:-}" ]; then
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$i -o run \
        --output-format csv -- python3 $R/bench.py $a --no-cpu-baseline > $OUT/bench_prof_$i.json 2> $OUT/bench_prof_$i.err ) \
      || { tail -20 $OUT/bench_prof_$i.err; exit 1; }
  fi
done
echo done
