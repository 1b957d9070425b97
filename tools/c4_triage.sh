for m in 1 4 64; do
  MSCCL_AMD_MERGE=$m MSCCL_AMD_TIMEOUT_SEC=5 timeout -k 10 100 python bench.py --no-cpu --quiet --steps 2 --warmup 1 --sizes 1048576 --extras C4 2>/dev/null | python -c "import json,sys; print('merge $m', json.load(sys.stdin).get('configs'))"
done
