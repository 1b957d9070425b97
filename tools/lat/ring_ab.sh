# ring fallback one-iteration calls: the small kernel against the general kernel, same box
set -o pipefail
run() { env $1 timeout -k 5 60 python3 tools/lat_one.py --iters 300 --graph --schedule fbring --bytes $2 --ranks $3 --dtype 6 $4 2>&1 | grep -v amdgpu.ids | sed "s|^|$1 |"; }
for rep in 1 2; do
  for e in MSCCL_AMD_SMALL_KERNEL=0 MSCCL_AMD_SMALL_KERNEL=1; do
    run $e 524288 8 || exit 1
    run $e 65536 8 || exit 1
    run $e 4096 8 || exit 1
    run $e 524288 2 || exit 1
    run $e 65536 8 "--coll rs" || exit 1
    run $e 65536 8 "--coll ag" || exit 1
  done
done
