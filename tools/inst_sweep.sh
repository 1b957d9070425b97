#!/bin/bash
# C2 pair-exchange instances x split over the upper half of the sweep (kernel us per size).
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
OUT=gpurun_out/inst
mkdir -p $OUT
: > $OUT/summary.txt
SZ=1048576,4194304,8388608,16777216,33554432
run() {  # name tiers env...
  local name=$1 tiers=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --no-cpu --quiet --steps 30 --warmup 5 --sizes $SZ --tiers $tiers > $OUT/$name.json 2>>$OUT/err.log || return 1
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('%-12s' % '$name', ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms']*1e3) for s in d['sweep']), 'ok' if d['verified'] else 'BAD')" >> $OUT/summary.txt
}
for I in 16; do run p$I 0:1073741825:$I:p || exit 1; done
run p16_s4 0:1073741825:16:p MSCCL_AMD_SPLIT=4 || exit 1
run p32_s4 0:1073741825:32:p MSCCL_AMD_SPLIT=4 || exit 1

run p16_t1024 0:1073741825:16:p MSCCL_AMD_TARGET_WGS=1024 || exit 1
cat $OUT/summary.txt
