#!/bin/bash
# The whole GPU suite, then the fallback at the new default thresholds (no size knob): AllReduce
# 64 / 256 / 512 KiB, ReduceScatter / AllGather 16 / 64 KiB per rank, 2 and 8 ranks, fp16.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03f}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_suite.txt 2>&1 || { tail -30 gpurun_out/${TAG}_suite.txt; exit 1; }
tail -1 gpurun_out/${TAG}_suite.txt
for n in 2 8; do
  for b in 65536 262144 524288; do
    timeout -k 5 60 python3 tools/lat_one.py --schedule fbtree --bytes $b --ranks $n --dtype 6 --iters 100 --graph 2>&1 \
      | grep -v amdgpu.ids | tee -a gpurun_out/${TAG}_defaults.txt || exit 1
  done
  for c in rs ag; do for b in 16384 65536; do
    timeout -k 5 60 python3 tools/lat_one.py --coll $c --schedule fbtree --bytes $b --ranks $n --dtype 6 --iters 100 \
      --graph 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${TAG}_defaults.txt || exit 1
  done; done
done
echo done
