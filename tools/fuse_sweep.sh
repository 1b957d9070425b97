#!/bin/bash
# Fused s + rrc exchange (MSCCL_AMD_FUSE) against the unfused schedule on
# the C2 pair tiers: kernel us per size, then FETCH_SIZE per 32 MiB launch (one PMC pass each).
set -o pipefail
export TMPDIR=/tmp MSCCL_AMD_TIMEOUT_SEC=20
OUT=gpurun_out/fuse
mkdir -p $OUT
: > $OUT/summary.txt
SZ=262144,1048576,4194304,16777216,33554432
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu --quiet --steps 30 --warmup 5 --sizes $SZ > $OUT/$name.json 2>>$OUT/err.log || return 1
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('%-10s' % '$name', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep']), 'ok' if d['verified'] else 'BAD')" >> $OUT/summary.txt
}
run unfused MSCCL_AMD_FUSE=0 || exit 1
run fused || exit 1
run unfused2 MSCCL_AMD_FUSE=0 || exit 1
run fused2 || exit 1
for V in 0 1; do
  MSCCL_AMD_FUSE=$V timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f$V -o run -- python3 bench.py --no-cpu --quiet --sizes 33554432 --steps 10 --warmup 2 > /dev/null 2>>$OUT/err.log || exit 1
  python3 - $OUT/f$V $V >> $OUT/summary.txt <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f))]
v = [float(r['Counter_Value']) for r in rows if 'mscclSmall' in r.get('Kernel_Name', '') and r['Counter_Name'] == 'FETCH_SIZE']
print('fuse=%s FETCH_SIZE per launch %.1f MB over %d dispatches' % (sys.argv[2], sum(v) / max(1, len(v)) * 1024 / 1e6, len(v)))
PY
done
cat $OUT/summary.txt
