#!/bin/bash
# Fold-kernel fallback latency per library (LIBS; same-box A/B when two are given): AllReduce /
# ReduceScatter / AllGather, 2 / 8 / 16 co-resident ranks, 128 B and 16 KiB per rank, fp16; the
# flat parity tests first.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03d}
OUT=gpurun_out/${TAG}_abfold
mkdir -p $OUT
: > $OUT/summary.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k flat > $OUT/flat_tests.txt 2>&1 || { tail -30 $OUT/flat_tests.txt; exit 1; }
tail -1 $OUT/flat_tests.txt
for rep in ${REPS:-1}; do for L in ${LIBS:-msccl_amd/libmsccl_amd.so}; do
  for c in ar rs ag; do for n in 2 8 16; do for b in 128 16384; do
    echo "rep$rep $(basename $L) $(MSCCL_AMD_LIB=$L timeout -k 5 60 python3 tools/lat_one.py --coll $c --schedule fbtree \
      --bytes $b --ranks $n --dtype 6 --iters 200 --graph 2>&1 | grep -v amdgpu.ids)" | tee -a $OUT/summary.txt || exit 1
  done; done; done
done; done
echo done
