#!/bin/bash
# Fallback latency (ring / chain tree / flat tree, device time from hipGraph replays), the C3 shape
# with C4 / C5 at 8 co-resident ranks and at 2, and rocprofv3 kernel-trace + PMC passes over the
# 8-rank configs (per-kernel traffic: tools/parse_prof.py).  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
RANKS="2 8" BYTES="128 4096 65536" bash tools/fb_sweep.sh > gpurun_out/${TAG}_fallback.txt 2>&1 || { tail -20 gpurun_out/${TAG}_fallback.txt; exit 1; }
cat gpurun_out/${TAG}_fallback.txt | grep -v amdgpu.ids
timeout -k 10 400 python3 bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
  > gpurun_out/${TAG}_c345_8.json 2> gpurun_out/${TAG}_c345_8.err || { tail -20 gpurun_out/${TAG}_c345_8.err; exit 1; }
timeout -k 10 400 python3 bench.py --vranks 2 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
  > gpurun_out/${TAG}_c45_2.json 2> gpurun_out/${TAG}_c45_2.err || { tail -20 gpurun_out/${TAG}_c45_2.err; exit 1; }
if [ -z "$SKIP_PROFILE" ]; then
  bash tools/profile.sh ${TAG}_extras8 --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
    > gpurun_out/${TAG}_prof_extras8.txt 2>&1 || { tail -20 gpurun_out/${TAG}_prof_extras8.txt; exit 1; }
fi
echo done
