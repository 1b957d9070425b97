set -o pipefail
mkdir -p /tmp/old && tar -xf ab_old.tar -C /tmp/old && (cd /tmp/old && timeout -k 10 400 make -C msccl_amd/csrc -j16 > /tmp/old_build.log 2>&1) || { tail -20 /tmp/old_build.log; exit 1; }
for i in 1 2; do
  for v in /tmp/old .; do
    timeout -k 10 100 python $v/bench.py --no-cpu --quiet --sizes 33554432 --steps 50 --warmup 10 | python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['roofline']['kernel_ms'])" || exit 1
  done
done
