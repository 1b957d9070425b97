# XCD grouping of thread blocks that send the same source (MSCCL_AMD_XCD_GROUP) with device-scope
# (sc1, the main build) and plain source loads (libvar_plain.so), 8 co-resident ranks (graph replay)
set -o pipefail
run() { env MSCCL_AMD_XCD_GROUP=$2 MSCCL_AMD_LIB=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 50 --graph "${@:3}" 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $1) xcd=$2 |"; }
for rep in 1 2; do for L in msccl_amd/libmsccl_amd.so tools/lat/libvar_plain.so; do for X in 0 1; do
  run $L $X --schedule agap --bytes 8388608 --ranks 8 --instances 8 --dtype 7 --proto Simple --coll ag || exit 1
  run $L $X --schedule rsap --bytes 8388608 --ranks 8 --instances 8 --dtype 7 --proto Simple --coll rs || exit 1
  run $L $X --schedule allpairs --bytes 33554432 --ranks 8 --instances 8 --dtype 6 || exit 1
done; done; done
