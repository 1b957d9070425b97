#!/bin/bash
# perf exploration on one MI355X: C2 shape (2 co-resident ranks), instances x sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
probe() {
  echo "== $*"
  timeout -k 10 120 env "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (s['bytes'], s['busbw'], s['kernel_ms']) for s in d['sweep']])" || exit 1
}
B="python bench.py --no-cpu --quiet --steps 40 --warmup 10 --sizes 65536,262144,1048576,4194304"
for i in 1 2 4 8 16; do
probe X=1 $B --instances $i
done
B="python bench.py --no-cpu --quiet --steps 40 --warmup 10 --sizes 128,4096,32768"
probe X=1 $B
probe MSCCL_AMD_TARGET_WGS=64 $B
