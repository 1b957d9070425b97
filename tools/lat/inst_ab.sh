# pair-exchange instances and workgroup budget at 4 / 16 / 32 MiB, one-pass pair calls (graph replay)
set -o pipefail
run() { env $1 timeout -k 5 120 python3 tools/lat_one.py --iters 100 --graph "${@:2}" 2>&1 | grep -v amdgpu.ids | sed "s|^|$1 |"; }
for rep in 1 2; do
  for cfg in "X=0 16" "X=0 32" "MSCCL_AMD_TARGET_WGS=512 32" "X=0 8" "MSCCL_AMD_TARGET_WGS=128 16"; do
    set -- $cfg
    for b in 4194304 16777216 33554432; do run $1 --schedule pair --bytes $b --ranks 2 --instances $2 --dtype 7 || exit 1; done
  done
done
