# GPU box: camera-phase tests, then the CAM bench under rocprofv3 --stats (kernel table printed).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/cam
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cam/pytest.log 2>&1 || { tail -40 gpurun_out/cam/pytest.log; exit 1; }
tail -2 gpurun_out/cam/pytest.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/cam/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cam/prof -o run --output-format csv -- python3 $R/bench.py --config CAM --steps 20 --warmup 5 ${CAM_ARGS:---no-cpu-baseline} > $R/gpurun_out/cam/bench.json 2> $R/gpurun_out/cam/bench.err || { tail -20 $R/gpurun_out/cam/bench.err; exit 1; }
cat $R/gpurun_out/cam/bench.json
python3 -c "import csv,sys; [print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:80]}\") for r in list(csv.DictReader(open(sys.argv[1])))[:12]]" $R/gpurun_out/cam/prof/run_kernel_stats.csv
