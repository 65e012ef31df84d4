# GPU box, one iteration: the gpu suite (or the pytest selection given), the default bench, and the
# bench under rocprofv3 --kernel-trace --stats (top kernels printed).  Usage: bash tools/experiments/gpu_iter.sh [TAG] [pytest args]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-it}; shift
O=gpurun_out/$TAG
mkdir -p $O
SEL=${@:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('ms/step',round(d['ms_per_step'],4),'stages',{k:round(v,4) for k,v in d['stage_ms'].items()})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/bench_prof.err || { tail -20 $R/$O/bench_prof.err; exit 1; }
F=$(find $R/$O/prof -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$F')))
for r in rows[:14]: print(f\"{float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}\")
"
