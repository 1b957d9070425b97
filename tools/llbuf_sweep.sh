#!/bin/bash
# LL FIFO slot size (NCCL_LL_BUFFSIZE / 8 per slot) on the C2 pair tiers: kernel us per size.
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
OUT=gpurun_out/llbuf
mkdir -p $OUT
: > $OUT/summary.txt
SZ=1048576,4194304,16777216,33554432
for B in 524288 262144 131072 1048576; do
  NCCL_LL_BUFFSIZE=$B timeout -k 10 120 python bench.py --no-cpu --quiet --steps 30 --warmup 5 --sizes $SZ > $OUT/b$B.json 2>>$OUT/err.log || exit 1
  python -c "import json; d=json.load(open('$OUT/b$B.json')); print('%-8s' % '$B', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep']), 'ok' if d['verified'] else 'BAD')" >> $OUT/summary.txt
done
cat $OUT/summary.txt
