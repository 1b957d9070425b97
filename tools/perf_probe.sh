#!/bin/bash
# perf exploration on one MI355X: C2 shape (2 co-resident ranks), knobs x sizes, 2 passes
set -o pipefail
cd $GRAFT_REPO_ROOT
probe() {
  echo "== $*"
  timeout -k 10 120 env "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (s['bytes'], s['busbw'], s['kernel_ms']) for s in d['sweep']], d['roofline']['achieved'])" || exit 1
}
B="python bench.py --no-cpu --quiet --steps 40 --warmup 10 --sizes 65536,1048576,4194304,8388608,16777216,33554432"
for pass in 1 2; do
probe X=1 $B --instances 16
probe X=1 $B --instances 16 --proto Simple
done
