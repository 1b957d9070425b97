set -o pipefail
run() { MSCCL_AMD_PAIR_KERNEL=$1 timeout -k 5 60 python3 tools/lat_one.py --iters 300 --graph --schedule pair --bytes $2 --ranks 2 --instances $3 2>&1 | grep -v amdgpu.ids | sed "s|^|pair=$1 |"; }
run 1 8192 16 || exit 1
for rep in 1 2 3; do for K in 0 1; do
  run $K 8192 16 || exit 1; run $K 65536 16 || exit 1; run $K 1048576 16 || exit 1; run $K 4194304 16 || exit 1
done; done
