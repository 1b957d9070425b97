# small-message latency: events per launch + rocprofv3 kernel duration, per schedule
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/latchk
for s in pair allpairs; do
  timeout -k 5 60 python3 tools/lat_one.py --schedule $s --bytes 128 >> gpurun_out/latchk/events.txt 2>&1 || exit 1
done
timeout -k 5 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/latchk/prof -o run -- python3 tools/lat_one.py --schedule pair --bytes 128 > gpurun_out/latchk/prof.log 2>&1 || exit 1
MSCCL_AMD_TRACE=1 timeout -k 5 60 python3 tools/trace_report.py --schedule pair --bytes 128 --iters 50 > gpurun_out/latchk/trace.txt 2>&1 || exit 1
