#!/bin/bash
# Where the one-hop fold kernel stops beating the ring: AllReduce (total bytes) and ReduceScatter /
# AllGather (bytes per rank's block), 2 / 8 / 16 co-resident ranks, fp16, ring vs the fold kernel
# with no size limit (MSCCL_AMD_TREE_MAX_BYTES=1 GiB), hipGraph replay.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03e}
OUT=gpurun_out/${TAG}_xover
mkdir -p $OUT
: > $OUT/summary.txt
for c in ${COLLS:-ar rs ag}; do for n in ${RANKS:-2 8 16}; do for b in ${BYTES:-65536 262144 1048576}; do
  for s in fbring fbtree; do
    echo "$(MSCCL_AMD_TREE_MAX_BYTES=1073741824 timeout -k 5 60 python3 tools/lat_one.py --coll $c --schedule $s \
      --bytes $b --ranks $n --dtype 6 --iters 100 --graph 2>&1 | grep -v amdgpu.ids)" | tee -a $OUT/summary.txt || exit 1
  done
done; done; done
echo done
