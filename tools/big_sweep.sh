#!/bin/bash
# 32 MiB C2 headline variants: pair one-shot instances x split / U (one bench line each)
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
mkdir -p gpurun_out/bs
: > gpurun_out/bs/summary.txt
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu --quiet --steps 30 --warmup 5 --sizes 33554432 $BARGS > gpurun_out/bs/$name.json 2>>gpurun_out/bs/err.log || return 1
  python -c "import json,sys; d=json.load(open('gpurun_out/bs/$name.json')); print('%-24s %8.1f GB/s  %7.2f us  frac %.3f' % ('$name', d['value'], d['sweep'][-1]['kernel_ms']*1e3, d['roofline']['frac']))" >> gpurun_out/bs/summary.txt
}
[ -n "$ONLY_SPLIT" ] || for I in 8 16 32; do
  BARGS="--tiers 0:1073741825:$I:p" run p$I MSCCL_AMD_X=0 || exit 1
done
for S in 2 4; do
  BARGS="--tiers 0:1073741825:16:p" run p16_split$S MSCCL_AMD_SPLIT=$S || exit 1
done
BARGS="--tiers 0:1073741825:32:p" run p32_split4 MSCCL_AMD_SPLIT=4 || exit 1
BARGS="--tiers 0:1073741825:16:p" run p16_split8 MSCCL_AMD_SPLIT=8 || exit 1
