# r06u: 2 rank processes on one GPU, every peer remote (the driver's --gpus 2 code paths): C2
# through the all-pairs XML tiers (lowered: the pair exchange) against the pair one-shot tiers
# (bench.PAIR_TIERS, rounds 2-5) and the all-pairs XML interpreted (MSCCL_AMD_LOWER_LARGE=0),
# 1 / 8 / 32 MiB, alternating, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
run() {  # tag env... -- args
  local tag=$1; shift
  env MSCCL_AMD_BENCH_ONE_GPU=1 MSCCL_AMD_FORCE_REMOTE=1 "$@" timeout -k 10 300 python bench.py --gpus 2 \
    --sizes 1048576,8388608,33554432 --steps 20 --warmup 5 --no-tuning --extras "" --no-secondary --pmc off \
    $EXTRA > $O/r06u.json 2>> $O/r06u.err || return 1
  python -c "
import json; d = json.load(open('$O/r06u.json'))
print('$tag', d['verified'], ' '.join('%d:%.1fus/%s' % (s['bytes'], s['ms'] * 1e3, s['kernel'][5:14]) for s in d['sweep']))" | tee -a $O/r06u_remote_pair.txt
}
for r in 1 2; do
  EXTRA="" run allpairs_lowered &&
  EXTRA="--tiers 0:4096:1:p,4096:1073741825:16:p" run pair_oneshot &&
  EXTRA="" run allpairs_interp MSCCL_AMD_LOWER_LARGE=0 || exit 1
done
