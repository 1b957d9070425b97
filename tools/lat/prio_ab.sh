# s_setprio 1 for the second half of a launch's workgroups (the later-dispatched workgroup of each CU)
set -o pipefail
run() { env $2 MSCCL_AMD_LIB=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 100 --graph "${@:3}" 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $1) $2 |"; }
for rep in 1 2; do for L in tools/lat/libvar_p0.so tools/lat/libvar_p1.so; do
  run $L MSCCL_AMD_TARGET_WGS=512 --schedule allpairs --bytes 16777216 --ranks 4 --instances 8 --dtype 7 || exit 1
  run $L MSCCL_AMD_TARGET_WGS=512 --schedule allpairs --bytes 33554432 --ranks 4 --instances 8 --dtype 7 || exit 1
  run $L X=0 --schedule allpairs --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
  run $L X=0 --schedule allpairs --bytes 33554432 --ranks 8 --instances 8 --dtype 7 || exit 1
  run $L X=0 --schedule allpairs --bytes 4194304 --ranks 8 --instances 8 --dtype 7 || exit 1
  run $L X=0 --schedule pair --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
done; done
