# kernel durations (rocprofv3) of small launches, traced and untraced
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/latprof
for tr in 0 1; do
  MSCCL_AMD_TRACE=$tr timeout -k 5 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/latprof/t$tr -o run -- python3 tools/lat_one.py --schedule pair --bytes 128 > gpurun_out/latprof/t$tr.log 2>&1 || exit 1
done
