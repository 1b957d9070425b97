# 2-rank schedule comparison over the whole sweep (one bench line per schedule)
set -o pipefail
export MSCCL_AMD_TIMEOUT_SEC=20
mkdir -p gpurun_out/ts2
for T in default 0:1073741825:1:p 0:1073741825:4:p 0:1073741825:16:p 0:1073741825:8:r 0:1073741825:16:r 0:1073741825:32:r 0:1073741825:16:a; do
  if [ "$T" = default ]; then A=""; else A="--tiers $T"; fi
  timeout -k 10 150 python bench.py --no-cpu --quiet --steps 20 --warmup 5 $A > gpurun_out/ts2/$(echo $T | tr ':' '_').json 2>gpurun_out/ts2/err.log || exit 1
done
