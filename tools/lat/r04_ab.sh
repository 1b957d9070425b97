# the round-4 library (tools/lat/libr04.so, built from e034aad) against the current one, same box:
# C3's 32 MiB all-pairs x8 (8 ranks fp16), C2's 32 MiB pair x16, C5's ReduceScatter x8 (graph replay)
set -o pipefail
run() { MSCCL_AMD_LIB=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 100 --graph "${@:2}" 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $1) |"; }
for rep in 1 2 3; do for L in tools/lat/libr04.so msccl_amd/libmsccl_amd.so; do
  run $L --schedule allpairs --bytes 33554432 --ranks 8 --instances 8 --dtype 6 || exit 1
  run $L --schedule pair --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
  run $L --schedule rsap --bytes 8388608 --ranks 8 --instances 8 --dtype 7 --proto Simple --coll rs || exit 1
done; done
