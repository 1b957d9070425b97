#!/bin/bash
# Flat ReduceScatter / AllGather (fold kernel): their parity tests, the ring fallback tests, then
# latency per launch, ring vs flat, per rank's block of 128 B / 4 KiB / 16 KiB, 2/4/8/16 ranks.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03c}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_ring.txt 2>&1 || { tail -30 gpurun_out/${TAG}_ring.txt; exit 1; }
tail -1 gpurun_out/${TAG}_ring.txt
for c in rs ag; do for n in ${RANKS:-2 4 8 16}; do for b in ${BYTES:-128 4096 16384}; do for s in fbring fbtree; do
  timeout -k 5 60 python3 tools/lat_one.py --coll $c --schedule $s --bytes $b --ranks $n --dtype 6 --iters 200 --graph \
    2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${TAG}_rsag_lat.txt || exit 1
done; done; done; done
if [ -n "$SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_suite.txt 2>&1 || { tail -30 gpurun_out/${TAG}_suite.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_suite.txt
fi
echo done
