#!/bin/bash
# perf exploration on one MI355X: C2 shape (2 co-resident ranks) at 1/8/32 MiB, protocol x instances x knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
probe() {
  echo "== $*"
  timeout -k 10 120 env "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (s['bytes'], s['busbw']) for s in d['sweep']], d['roofline']['achieved'])" || exit 1
}
B="python bench.py --no-cpu --quiet --steps 20 --warmup 5 --sizes 1048576,8388608,33554432"
probe X=1 $B --instances 16
probe X=1 $B --instances 32
probe MSCCL_AMD_ARENA_COARSE=1 $B --instances 16
probe MSCCL_AMD_TARGET_WGS=512 $B --instances 16
probe MSCCL_AMD_TARGET_WGS=1024 $B --instances 16
probe MSCCL_AMD_MERGE=1 $B --instances 16
probe X=1 $B --proto Simple --instances 16
probe MSCCL_AMD_ARENA_COARSE=1 $B --proto Simple --instances 16
probe MSCCL_AMD_TARGET_WGS=512 $B --proto Simple --instances 16
probe X=1 $B --vranks 8 --instances 4
