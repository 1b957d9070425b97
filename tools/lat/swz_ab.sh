# grid halves interleaved in the small kernel (libvar_swz.so, MSCCL_BLOCK_SWIZZLE) against the main
# build: 8-rank C3 32 MiB (512 workgroups) and the 4-rank 16 MiB call at 512 workgroups
set -o pipefail
run() { env $2 MSCCL_AMD_LIB=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 50 --graph "${@:3}" 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $1) $2 |"; }
for rep in 1 2; do for L in msccl_amd/libmsccl_amd.so tools/lat/libvar_swz.so; do
  run $L X=0 --schedule allpairs --bytes 33554432 --ranks 8 --instances 8 --dtype 6 || exit 1
  run $L MSCCL_AMD_TARGET_WGS=512 --schedule allpairs --bytes 16777216 --ranks 4 --instances 8 --dtype 7 || exit 1
  run $L X=0 --schedule allpairs --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
done; done
