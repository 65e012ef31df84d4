# GPU box: A/B of experiment libraries (tools/exp_variants.py builds loner_amd/_lib/variants/<tag>.so)
# against the default library: the bench line's stage times per library (REP rounds, interleaved),
# then the training digest of each (tools/lib_digest.py: a variant must change no bit).
#   bash tools/gpu_ab_libs.sh "tag1 tag2 ..." ["<bench args>"]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/ablib
mkdir -p $OUT
REP=${REP:-2}
ARGS=${2:-}
libs="default $1"
libpath() { [ "$1" = default ] && echo $R/loner_amd/_lib/libloner_amd.so || echo $R/loner_amd/_lib/variants/$1.so; }
for rep in $(seq $REP); do
  for t in $libs; do
    LONER_AMD_LIB=$(libpath $t) timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline > $OUT/b_$t.json 2> $OUT/b_$t.err \
      || { tail -20 $OUT/b_$t.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/b_$t.json').read().strip().splitlines()[-1]); s=d['stage_ms']
print(f'[$t] {d[\"ms_per_step\"]:.4f} ms  ' + ' '.join(f'{k}={v:.4f}' for k,v in s.items()), flush=True)"
  done
done
for t in $libs; do
  LONER_AMD_LIB=$(libpath $t) timeout -k 10 120 python tools/lib_digest.py 3 > $OUT/d_$t.txt 2>&1 || { tail -20 $OUT/d_$t.txt; exit 1; }
  echo "[$t] $(tail -1 $OUT/d_$t.txt)"
done
echo ablib done
