set -o pipefail
B="python bench.py --no-cpu --quiet --steps 50 --warmup 10 --sizes 128,65536,1048576,8388608,33554432"
for v in 0 1 0 1; do
  MSCCL_AMD_ARENA_COARSE=$v timeout -k 10 100 $B 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('coarse=$v', [(s['bytes'], s['busbw'], s.get('kernel_ms')) for s in d['sweep']])" || exit 1
done
MSCCL_AMD_ARENA_COARSE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "allpairs_allreduce or ring or split" 2>&1 | tail -3
