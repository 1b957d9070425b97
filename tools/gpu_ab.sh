#!/bin/bash
# Same-box A/B runs (box-to-box variation is up to 10 %, so only same-box pairs compare):
#   fold kernel workgroups per rank (MSCCL_AMD_FOLD_WGS=1 vs the default) on the flat tree's sizes;
#   the round-2 library (MSCCL_AMD_LIB=tools/ab/libmsccl_amd_r02.so) vs this tree on the C2 and C3
#   32 MiB launches and the 2-rank 128 B pair latency.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03c}
OUT=gpurun_out/${TAG}_ab
mkdir -p $OUT
: > $OUT/summary.txt
lat() { timeout -k 5 60 python3 tools/lat_one.py --iters 200 --graph "$@" 2>&1 | grep -v amdgpu.ids; }
for W in ${FOLD_WGS-1 4}; do
  for n in 2 8 16; do for b in 128 4096 16384; do
    echo "wgs<=$W $(MSCCL_AMD_FOLD_WGS=$W lat --schedule fbtree --bytes $b --ranks $n --dtype 6)" | tee -a $OUT/summary.txt || exit 1
  done; done
done
for L in ${LIBS:-tools/ab/libmsccl_amd_r02.so msccl_amd/libmsccl_amd.so}; do
  echo "lib $L: $(MSCCL_AMD_LIB=$L lat --schedule pair --bytes 128 --ranks 2)" | tee -a $OUT/summary.txt || exit 1
  MSCCL_AMD_LIB=$L timeout -k 10 300 python3 bench.py --sizes 33554432 --no-cpu --pmc off --no-secondary > $OUT/c2_$(basename $L).json 2>>$OUT/err.log || exit 1
  MSCCL_AMD_LIB=$L timeout -k 10 300 python3 bench.py --vranks 8 --dtype fp16 --sizes 33554432 --no-cpu --pmc off --no-secondary > $OUT/c3_$(basename $L).json 2>>$OUT/err.log || exit 1
  python3 -c "import json; a=json.load(open('$OUT/c2_$(basename $L).json')); b=json.load(open('$OUT/c3_$(basename $L).json')); print('lib $L: C2 32 MiB %.1f GB/s kernel %.4f ms | C3 32 MiB %.1f GB/s kernel %.4f ms' % (a['value'], a['sweep'][-1]['kernel_ms'], b['value'], b['sweep'][-1]['kernel_ms']))" | tee -a $OUT/summary.txt
done
echo done
