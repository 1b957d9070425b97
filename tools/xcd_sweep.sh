#!/bin/bash
# Placement experiments on the C2 headline (2 co-resident ranks, pair tiers, 32 MiB):
# MSCCL_AMD_FIFO_PAD bytes after every FIFO (so sub-connections do not share an offset modulo the
# FIFO size): kernel us per size, then the light trace's per-XCD finish times (the XCD each
# workgroup ran on comes from HW_REG_XCC_ID).  The rank-rotation experiment (rank 1's workgroups
# shifted by K grid slots) is recorded in profiles/r03_xcd_placement.txt; its knob was not kept.  (The round-2
# chunk-skew experiment this script once ran is recorded in profiles/r02_xcd_skew_sweep.txt; its
# knob was not kept.)
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
OUT=${OUT:-gpurun_out/xcd}
mkdir -p $OUT
: > $OUT/summary.txt
SZ=${SZ:-4194304,16777216,33554432}
PADS=${PADS:-"0 4096 65536 200704 0"}
for P in $PADS; do
  MSCCL_AMD_FIFO_PAD=$P timeout -k 10 120 python bench.py --no-cpu --quiet --no-secondary --pmc off --steps 30 --warmup 5 --sizes $SZ > $OUT/p$P.json 2>>$OUT/err.log || exit 1
  python -c "import json; d=json.load(open('$OUT/p$P.json')); print('pad %-7s' % '$P', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep']), 'ok' if d['verified'] else 'BAD')" >> $OUT/summary.txt
done
for P in ${TRACE_PADS:-0 4096}; do
  MSCCL_AMD_FIFO_PAD=$P MSCCL_AMD_TRACE=2 timeout -k 10 120 python tools/trace_report.py --bytes 33554432 --instances 16 --schedule pair --iters 10 > $OUT/trace$P.txt 2>&1 || exit 1
  python - $OUT/trace$P.txt $P >> $OUT/summary.txt <<'PY'
import re, sys
import numpy as np
rows = []
for l in open(sys.argv[1]):
    m = re.search(r'slot\s+(\d+): start ([\d.]+) \| done ([\d.]+) xcc (\d+)', l)
    if m:
        rows.append((int(m.group(4)), float(m.group(3))))
a = np.array(rows)
x = [a[a[:, 0] == k, 1].mean() for k in range(8)]   # by the XCD the workgroup ran on (HW_REG_XCC_ID)
print('pad %s: done median %.1f max %.1f; per-XCD mean %s' % (sys.argv[2], np.median(a[:, 1]), a[:, 1].max(), ' '.join('%.1f' % v for v in x)))
PY
done
cat $OUT/summary.txt
