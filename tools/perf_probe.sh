#!/bin/bash
# perf exploration on one MI355X: instance counts / protocols at 32 MiB, C2 shape
set -o pipefail
cd $GRAFT_REPO_ROOT
for args in "--instances 16" "--instances 32" "--proto Simple --instances 16" "--proto Simple --instances 32" "--vranks 8 --instances 4" "--vranks 8 --instances 4 --proto Simple"; do
  echo "== $args"
  timeout -k 10 120 python bench.py --no-cpu --quiet --steps 20 --warmup 5 --sizes 1048576,8388608,33554432 $args | python -c "import json,sys; d=json.loads(sys.stdin.read()); print([ (s['bytes'], s['busbw']) for s in d['sweep']], d['roofline']['achieved'])" || exit 1
done
