# r06o: the driver's multi-GPU bench commands rehearsed on one GPU with every peer treated as remote
# (MSCCL_AMD_FORCE_REMOTE=1: the cross-GPU tiers, limits, fences and the 4 MiB Simple FIFO), with
# the tuning keys: 8 and 2 rank processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
MSCCL_AMD_BENCH_ONE_GPU=1 MSCCL_AMD_FORCE_REMOTE=1 timeout -k 10 600 python bench.py --gpus 8 --steps 20 --warmup 5 \
  > $O/r06o_rehearse_8_remote.json 2> $O/r06o_rehearse_8_remote.err &&
MSCCL_AMD_BENCH_ONE_GPU=1 MSCCL_AMD_FORCE_REMOTE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 \
  > $O/r06o_rehearse_2_remote.json 2> $O/r06o_rehearse_2_remote.err
