#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 4 8 16; do
  MSCCL_AMD_BENCH_C5_INSTANCES=$i timeout -k 10 200 python bench.py --no-cpu --quiet --steps 10 --warmup 3 --sizes 1048576 --extras C4,C5 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print($i, d['configs'])" || exit 1
done
