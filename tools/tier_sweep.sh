set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
S=1048576,2097152,4194304,8388608,16777216,33554432
for T in 0:1073741825:16:o 0:1073741825:32:o 0:1073741825:4:o 0:1073741825:32:a 0:1073741825:8:a; do
  timeout -k 10 120 python bench.py --no-cpu --quiet --sizes $S --tiers $T > gpurun_out/ts_$T.json 2>/dev/null || exit 1
done
