# r06t: 8 rank processes on one GPU with every peer treated as remote (the driver's 8-GPU code
# paths), the C3 shape at 1 / 8 / 32 MiB: lowered large calls (two-phase fold) against the
# interpreted schedule (MSCCL_AMD_LOWER_LARGE=0), alternating, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for L in 1 0; do
    MSCCL_AMD_LOWER_LARGE=$L MSCCL_AMD_BENCH_ONE_GPU=1 MSCCL_AMD_FORCE_REMOTE=1 timeout -k 10 300 python bench.py --gpus 8 \
      --sizes 1048576,8388608,33554432 --steps 20 --warmup 5 --no-tuning --extras "" --no-secondary --pmc off \
      > $O/r06t.json 2>> $O/r06t.err || exit 1
    python -c "
import json; d = json.load(open('$O/r06t.json'))
print('LOWER_LARGE=$L', d['verified'], ' '.join('%d:%.1fus/%s' % (s['bytes'], s['ms'] * 1e3, s['kernel'][5:14]) for s in d['sweep']))" | tee -a $O/r06t_remote_lowered.txt
  done
done
