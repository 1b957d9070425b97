# the lowered fold against the pair kernel on the 2-rank pair schedule, 128 B - 8 KiB (graph replay)
set -o pipefail
run() { env $1 timeout -k 5 60 python3 tools/lat_one.py --iters 300 --graph --schedule pair --bytes $2 --ranks 2 --instances $3 2>&1 | grep -v amdgpu.ids | sed "s|^|$1 |"; }
run MSCCL_AMD_LOWER=1 128 1 || exit 1
for rep in 1 2; do for b in 128 1024 4096 8192; do for inst in 1 16; do
  run MSCCL_AMD_LOWER_MAX_BYTES=65536 $b $inst || exit 1
  run MSCCL_AMD_LOWER=0 $b $inst || exit 1
done; done; done
