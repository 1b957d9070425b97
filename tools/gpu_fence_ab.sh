#!/bin/bash
# Simple hand-off: the sc0 sc1 form (default) against agent-scope fences on local connections
# (MSCCL_AMD_SIMPLE_FENCE=1), on the C4 / C5 shapes at 2 co-resident ranks; ReduceScatter chain
# against scratch form at 8; the 8-rank C3 shape over the whole sweep.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
: > gpurun_out/${TAG}_fence_ab.txt
for F in 0 1 0 1; do
  MSCCL_AMD_SIMPLE_FENCE=$F timeout -k 10 300 python3 bench.py --vranks 2 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
    > gpurun_out/${TAG}_fence$F.json 2>>gpurun_out/${TAG}_fence_ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_fence$F.json').read().strip().splitlines()[-1]); c=d['configs']; print('fence $F: C4 %.1f  RS %.1f  AG %.1f GB/s' % (c['C4']['allreduce']['busbw'], c['C5']['reduce_scatter']['busbw'], c['C5']['all_gather']['busbw']), c['C4']['verified'], c['C5']['verified'])" >> gpurun_out/${TAG}_fence_ab.txt
done
for FORM in chain scratch; do
  MSCCL_AMD_BENCH_RS_FORM=$FORM timeout -k 10 300 python3 bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C5 --no-cpu --pmc off --no-secondary \
    > gpurun_out/${TAG}_rs8_$FORM.json 2>>gpurun_out/${TAG}_fence_ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_rs8_$FORM.json').read().strip().splitlines()[-1]); c=d['configs']['C5']; print('8 ranks RS $FORM: %.1f GB/s (kernel %.3f ms, hbm frac %.3f)  AG %.1f' % (c['reduce_scatter']['busbw'], c['reduce_scatter']['kernel_ms'], c['reduce_scatter']['hbm_frac'], c['all_gather']['busbw']), c['verified'])" >> gpurun_out/${TAG}_fence_ab.txt
done
timeout -k 10 400 python3 bench.py --vranks 8 --dtype fp16 --no-cpu --pmc off --no-secondary > gpurun_out/${TAG}_c3_sweep.json 2>>gpurun_out/${TAG}_fence_ab.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_c3_sweep.json').read().strip().splitlines()[-1]); print('C3 shape sweep: 32 MiB %.1f GB/s kernel %.3f ms; 128 B %.2f us' % (d['value'], d['roofline']['kernel_ms'], d['sweep'][0]['kernel_ms']*1e3), d['verified'])" >> gpurun_out/${TAG}_fence_ab.txt
cat gpurun_out/${TAG}_fence_ab.txt
