# MSCCL_AMD_RUN_SLOTS 4 (default) against 8: merged runs of sends up to the whole FIFO, the
# Simple C5 pair, the C4 ring and LL C3 / 2-rank two-phase (graph replay, 8 co-resident ranks)
set -o pipefail
run() { env MSCCL_AMD_TIMEOUT_SEC=20 MSCCL_AMD_RUN_SLOTS=$1 timeout -k 5 120 python3 tools/lat_one.py --iters 30 --graph "${@:2}" 2>&1 | grep -v amdgpu.ids | sed "s|^|slots=$1 |"; }
for rep in 1 2; do for S in 4 8; do
  run $S --schedule agap --bytes 8388608 --ranks 8 --instances 8 --dtype 7 --proto Simple --coll ag || exit 1
  run $S --schedule rsap --bytes 8388608 --ranks 8 --instances 8 --dtype 7 --proto Simple --coll rs || exit 1
  run $S --schedule ring --bytes 268435456 --ranks 8 --instances 32 --dtype 9 --proto Simple || exit 1
  run $S --schedule allpairs --bytes 33554432 --ranks 8 --instances 8 --dtype 6 || exit 1
  run $S --schedule allpairs --bytes 33554432 --ranks 2 --instances 16 --dtype 7 || exit 1
done; done
