#!/bin/bash
# Same-box A/B of the kernel-argument warm-up + one-round-trip prologue (tools/ab/libmsccl_amd_new.so:
# this tree's fp32 kernels) against the committed build, and the latency trace of both.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03e_warm
mkdir -p $OUT
for L in msccl_amd/libmsccl_amd.so tools/ab/libmsccl_amd_new.so msccl_amd/libmsccl_amd.so tools/ab/libmsccl_amd_new.so; do
  for s in pair fbtree; do
    echo "$L $(MSCCL_AMD_LIB=$L timeout -k 5 60 python3 tools/lat_one.py --schedule $s --bytes 128 --ranks 2 --dtype 7 --iters 200 --graph 2>&1 | grep -v amdgpu.ids)" | tee -a $OUT/summary.txt || exit 1
  done
  MSCCL_AMD_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --pmc off --no-secondary > $OUT/bench_$(basename $L).json 2>>$OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_$(basename $L).json')); print('$L sweep', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep'] if s['bytes'] in (128, 4096, 65536, 1048576, 33554432)), 'value %.1f avg %.1f' % (d['value'], d['avg_busbw']))" | tee -a $OUT/summary.txt
done
for L in tools/ab/libmsccl_amd_lat.so tools/ab/libmsccl_amd_lat2.so; do
  echo "== $L" | tee -a $OUT/summary.txt
  MSCCL_AMD_LIB=$L MSCCL_AMD_TRACE=2 timeout -k 10 120 python3 tools/lat_trace.py 128 2>&1 | grep -v amdgpu.ids | grep "rank 0" | tee -a $OUT/summary.txt || exit 1
done
echo done
