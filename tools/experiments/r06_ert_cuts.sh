set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6t3
ERT_SWEEP=cuts timeout -k 10 800 python -u tools/experiments/r06_ert_tmin.py > gpurun_out/r6t3/log.txt 2>&1; tail -14 gpurun_out/r6t3/log.txt
