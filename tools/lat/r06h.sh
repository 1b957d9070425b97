# r06h: the C2 sweep through the msccl-tools two-phase all-pairs tiers with the 2-rank fold limit
# at its default (4 KiB) and at 0 (every call the lowered pair kernel), driver form; C4 / C5 with
# the direct kernel's per-collective workgroup defaults; the 8-process one-GPU rehearsal with the
# tuning keys timed by graph replay
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
BARGS="--tiers 0:4096:1:a,4096:1073741825:16:a --steps 20 --warmup 5" SWEEPENVS="-;MSCCL_AMD_LOWER_MAX_BYTES=0;-;MSCCL_AMD_LOWER_MAX_BYTES=0" \
  STEPS=envsweep TAG=r06h bash tools/gpu_session.sh &&
timeout -k 10 300 python bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
  --steps 10 --warmup 3 > $O/r06h_c45.json 2> $O/r06h_c45.err &&
MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 8 --steps 20 --warmup 5 \
  > $O/r06h_rehearse_8.json 2> $O/r06h_rehearse_8.err
