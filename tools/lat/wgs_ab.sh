# MSCCL_AMD_TARGET_WGS 256 against 512 for LL schedules with 2 and 4 co-resident ranks (graph replay)
set -o pipefail
run() { MSCCL_AMD_TARGET_WGS=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 100 --graph "${@:2}" 2>&1 | grep -v amdgpu.ids | sed "s|^|wgs=$1 |"; }
for rep in 1 2; do for W in 256 512; do
  run $W --schedule allpairs --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
  run $W --schedule allpairs --bytes 4194304 --ranks 2 --instances 16 --dtype 7 || exit 1
  run $W --schedule pair --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
  run $W --schedule allpairs --bytes 33554432 --ranks 4 --instances 8 --dtype 7 || exit 1
  run $W --schedule allpairs --bytes 1048576 --ranks 4 --instances 8 --dtype 7 || exit 1
  run $W --schedule allpairs --bytes 33554432 --ranks 4 --instances 4 --dtype 7 || exit 1
done; done
