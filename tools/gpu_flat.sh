#!/bin/bash
# Flat tree (fold kernel) session: its parity tests, the whole GPU suite, fallback latency per
# launch for 2/4/8/16 co-resident ranks, the per-XCD finish times of the C2 32 MiB launch.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03b}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k flat > gpurun_out/${TAG}_flat.txt 2>&1 || { tail -30 gpurun_out/${TAG}_flat.txt; exit 1; }
tail -1 gpurun_out/${TAG}_flat.txt
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_suite.txt 2>&1 || { tail -30 gpurun_out/${TAG}_suite.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_suite.txt
fi
RANKS="2 4 8 16" BYTES="128 4096 16384" bash tools/fb_sweep.sh 2>&1 | grep -v amdgpu.ids > gpurun_out/${TAG}_fallback.txt || exit 1
grep fbtree gpurun_out/${TAG}_fallback.txt
for F in 1 0; do   # C3 shape with and without the flat tree's connections (arena layout A/B)
  MSCCL_AMD_TREE_FLAT=$F timeout -k 10 300 python3 bench.py --vranks 8 --dtype fp16 --sizes 33554432 --no-cpu --pmc off \
    --no-secondary > gpurun_out/${TAG}_c3_flat$F.json 2> gpurun_out/${TAG}_c3_flat$F.err || { tail -5 gpurun_out/${TAG}_c3_flat$F.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_flat$F.json')); print('C3 32 MiB flat=$F', d['value'], d['sweep'][-1]['kernel_ms'])"
done
OUT=gpurun_out/${TAG}_xcd PADS=" " ROTS=" " TRACE_PADS="0" bash tools/xcd_sweep.sh > /dev/null 2>&1 || exit 1
cat gpurun_out/${TAG}_xcd/summary.txt
echo done
