# joint pose + map at C2: the d_pos launch shapes (passes vs one level-outer launch, samples per thread)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6dp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_input_grad.py tests/test_gpu_pose.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for spt in 2 0 4 8; do
  LONER_DPOS_SPT=$spt timeout -k 10 300 python bench.py --config C2 --joint-poses --no-cpu-baseline > $O/jp$spt.json 2>$O/jp$spt.err || exit 1
  python3 -c "import json; d=json.load(open('$O/jp$spt.json')); print('spt $spt', round(d['ms_per_step'],4), round(d['stage_ms']['pose_grad'],4), round(d['stage_ms']['pose_adam'],4))"
done
