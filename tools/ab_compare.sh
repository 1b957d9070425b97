# A/B: bench of the trees in ab_*.tar (built on the box) vs this tree, alternating, same box
set -o pipefail
SIZES=${1:-33554432}
TREES=""
for t in ab_*.tar; do
  d=/tmp/${t%.tar}
  mkdir -p $d && tar -xf $t -C $d && (cd $d && timeout -k 10 400 make -C msccl_amd/csrc -j16 > /tmp/build_${t%.tar}.log 2>&1) || { tail -20 /tmp/build_${t%.tar}.log; exit 1; }
  TREES="$TREES $d"
done
for i in 1 2; do
  for v in $TREES .; do
    timeout -k 10 100 python $v/bench.py --no-cpu --quiet --sizes $SIZES --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$v', [(s['bytes'], s['busbw'], s.get('kernel_ms')) for s in d['sweep']])" || exit 1
  done
done
