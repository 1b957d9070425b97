# 8 co-resident ranks on one MI355X, fp16 LL: two-phase all-pairs vs rank-ordered one-shot
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
S=128,1024,8192,65536,262144,1048576,4194304
for T in 0:1073741825:1:a 0:1073741825:1:O 0:1073741825:4:O; do
  timeout -k 10 120 python bench.py --no-cpu --quiet --vranks 8 --dtype fp16 --sizes $S --tiers $T > gpurun_out/ts8_$T.json 2>/dev/null || exit 1
done
