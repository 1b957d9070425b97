set -o pipefail
run() { MSCCL_AMD_LIB=$1 timeout -k 5 60 python3 tools/lat_one.py --iters 300 --graph --schedule pair --bytes $2 --ranks 2 --instances $3 2>&1 | grep -v amdgpu.ids | sed "s|^|$1 |"; }
run tools/lat/libvar_pin2.so 8192 16 || exit 1
for rep in 1 2 3; do for L in tools/lat/libvar_base.so tools/lat/libvar_pin2.so; do
  run $L 8192 16 || exit 1; run $L 1048576 16 || exit 1; run $L 4194304 16 || exit 1
done; done
