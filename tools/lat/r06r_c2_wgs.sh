# r06r: the C2 sweep (driver form) with the lowered pair's workgroups per rank at 64 (default flat
# budget 256) against 128 (MSCCL_AMD_TARGET_WGS=512), alternating, three rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for w in 256 512; do
    MSCCL_AMD_TARGET_WGS=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --pmc off --no-secondary \
      > $O/r06r_sw.json 2>> $O/r06r_sw.err || exit 1
    python -c "
import json; d = json.load(open('$O/r06r_sw.json'))
print('wgs$w', 'value %.1f avg %.2f |' % (d['value'], d['avg_busbw']), ' '.join('%d:%.2f' % (s['bytes'], s['kernel_ms'] * 1e3) for s in d['sweep']))" | tee -a $O/r06r_c2_wgs.txt
  done
done
