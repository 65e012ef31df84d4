# GPU box, round 4 evidence in one call: the whole -m gpu suite, the committed profile set for the
# configs given (bench line with cpu_baseline + rocprofv3 kernel stats, tools/gpu_r3_profiles.sh), then
# the parts of tools/gpu_r4.sh named in PARTS (calib pmc slack).
#   bash tools/gpu_r4_all.sh "C2 C1" "calib pmc slack"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -v -x --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/r4/suite.log 2>&1 || { tail -40 gpurun_out/r4/suite.log; exit 1; }
tail -1 gpurun_out/r4/suite.log
if [ -n "$1" ]; then PROF_DIR=r4p bash tools/gpu_r3_profiles.sh "$1" || exit 1; fi
if [ -n "$2" ]; then bash tools/gpu_r4.sh "$2" || exit 1; fi
echo all done
