#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
probe() {
  echo "== $*"
  timeout -k 10 120 env "$@" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (s['bytes'], s['busbw'], s['kernel_ms']) for s in d['sweep']])" || exit 1
}
B="python bench.py --no-cpu --quiet --steps 40 --warmup 10 --sizes 128,65536,1048576,8388608,33554432"
probe X=1 $B
probe X=1 $B
