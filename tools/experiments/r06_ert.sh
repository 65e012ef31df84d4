set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_live.py > $O/live.log 2>&1 || { tail -30 $O/live.log; exit 1; }
tail -1 $O/live.log
for spec in "C2" "C2 --joint-poses" ; do
  t=$(echo $spec | tr -d ' -')
  timeout -k 10 300 python bench.py --config $spec --no-cpu-baseline > $O/b_$t.json 2> $O/b_$t.err || { tail -5 $O/b_$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$t.json')); print('$t', round(d['ms_per_step'],4), d['stage_ms'])"
done
LONER_ERT=0 timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $O/b_C2noert.json 2> $O/b_C2noert.err || exit 1
python3 -c "import json; d=json.load(open('$O/b_C2noert.json')); print('C2noert', round(d['ms_per_step'],4), d['stage_ms'])"
