#!/bin/bash
# MSCCL_AMD_XCD_SKEW (permille more chunk positions for even-XCD workgroups) on the C2 pair
# tiers: kernel us per size, then the light trace's per-XCD finish times at 32 MiB.
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
OUT=gpurun_out/xcd
mkdir -p $OUT
: > $OUT/summary.txt
SZ=1048576,4194304,16777216,33554432
for K in 0 40 60 80 0; do
  MSCCL_AMD_XCD_SKEW=$K timeout -k 10 120 python bench.py --no-cpu --quiet --steps 30 --warmup 5 --sizes $SZ > $OUT/k$K.json 2>>$OUT/err.log || exit 1
  python -c "import json; d=json.load(open('$OUT/k$K.json')); print('%-4s' % '$K', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep']), 'ok' if d['verified'] else 'BAD')" >> $OUT/summary.txt
done
for K in 0 60; do
  MSCCL_AMD_XCD_SKEW=$K MSCCL_AMD_TRACE=2 timeout -k 10 120 python tools/trace_report.py --bytes 33554432 --instances 16 --schedule pair --iters 10 > $OUT/trace$K.txt 2>&1 || exit 1
  python - $OUT/trace$K.txt $K >> $OUT/summary.txt <<'PY'
import re, sys
import numpy as np
rows = []
for l in open(sys.argv[1]):
    m = re.search(r'slot\s+(\d+): start ([\d.]+) \| done ([\d.]+)', l)
    if m:
        rows.append((int(m.group(1)), float(m.group(3))))
a = np.array(rows)
even, odd = a[a[:, 0] % 2 == 0, 1], a[a[:, 0] % 2 == 1, 1]
print('skew %s: done median %.1f max %.1f; even-XCD mean %.1f, odd-XCD mean %.1f' % (sys.argv[2], np.median(a[:, 1]), a[:, 1].max(), even.mean(), odd.mean()))
PY
done
cat $OUT/summary.txt
