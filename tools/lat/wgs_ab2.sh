# MSCCL_AMD_TARGET_WGS 256 against 512, the mid sizes (graph replay)
set -o pipefail
run() { MSCCL_AMD_TARGET_WGS=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 100 --graph "${@:2}" 2>&1 | grep -v amdgpu.ids | sed "s|^|wgs=$1 |"; }
for rep in 1 2; do for W in 256 512; do
  for b in 8388608 16777216; do run $W --schedule allpairs --bytes $b --ranks 2 --instances 16 --dtype 7 || exit 1; done
  for b in 4194304 8388608 16777216; do run $W --schedule allpairs --bytes $b --ranks 4 --instances 8 --dtype 7 || exit 1; done
  run $W --schedule pair --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
done; done
