# 8 co-resident ranks on one MI355X, fp16 LL (C3 shape): schedule forms over the sweep
#   two-phase all-pairs (a) with 1 / 4 / 16 instances, rank-ordered one-shot (O) with 1 / 4, default tiers
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
mkdir -p gpurun_out/ts8
S=128,1024,8192,65536,262144,1048576,4194304,16777216,33554432
for T in ${TIERS:-default 0:1073741825:1:a 0:1073741825:4:a 0:1073741825:1:O 0:1073741825:4:O}; do
  if [ "$T" = default ]; then A=""; else A="--tiers $T"; fi
  timeout -k 10 150 python bench.py --no-cpu --quiet --vranks 8 --dtype fp16 --steps 20 --sizes $S $A > gpurun_out/ts8/$(echo $T | tr ':' '_').json 2>>gpurun_out/ts8/err.log || exit 1
done
