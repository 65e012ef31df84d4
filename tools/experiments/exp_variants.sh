# Run tools/exp_kernels.py under rocprofv3 --stats for the default build and every variant library
# under loner_amd/_lib/variants/ (GPU box).  Output: gpurun_out/exp/<tag>/...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
shopt -s nullglob
for lib in $R/loner_amd/_lib/libloner_amd.so $R/loner_amd/_lib/variants/*.so; do
  tag=$(basename $lib .so)
  mkdir -p $R/gpurun_out/exp/$tag
  LONER_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exp/$tag -o run \
    --output-format csv -- python3 $R/tools/exp_kernels.py > $R/gpurun_out/exp/$tag/out.txt 2>&1 || { echo "FAIL $tag"; tail -20 $R/gpurun_out/exp/$tag/out.txt; exit 1; }
  echo "$tag: $(tail -1 $R/gpurun_out/exp/$tag/out.txt)"
done
