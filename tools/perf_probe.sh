#!/bin/bash
# perf exploration on one MI355X: C2 shape (2 co-resident ranks), knobs x sizes, 2 passes
set -o pipefail
cd $GRAFT_REPO_ROOT
probe() {
  echo "== $*"
  timeout -k 10 120 env "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (s['bytes'], s['busbw']) for s in d['sweep']], d['roofline']['achieved'])" || exit 1
}
B="python bench.py --no-cpu --quiet --steps 40 --warmup 10 --sizes 1048576,8388608,33554432"
for pass in 1 2; do
probe X=1 $B --instances 16
probe X=1 $B --instances 32
probe X=1 $B --instances 16 --proto LL128
probe MSCCL_AMD_MERGE=4 $B --instances 16 --proto LL128
probe X=1 $B --instances 16 --proto Simple
probe MSCCL_AMD_MERGE=4 $B --instances 16 --proto Simple
probe X=1 $B --instances 8 --proto Simple
done
