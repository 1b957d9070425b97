#!/bin/bash
# C2 pair-exchange instance count over the small and mid sizes (kernel us per size).
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
OUT=gpurun_out/stier
mkdir -p $OUT
: > $OUT/summary.txt
SZ=128,1024,4096,16384,65536,262144,1048576
for I in 1 2 4 8 16; do
  timeout -k 10 120 python bench.py --no-cpu --quiet --steps 50 --warmup 10 --sizes $SZ --tiers 0:1073741825:$I:p > $OUT/i$I.json 2>>$OUT/err.log || exit 1
  python -c "import json; d=json.load(open('$OUT/i$I.json')); print('%-3s' % '$I', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep']), 'ok' if d['verified'] else 'BAD')" >> $OUT/summary.txt
done
cat $OUT/summary.txt
