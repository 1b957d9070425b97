#!/bin/bash
# One GPU session's checks, run from the repo root on the GPU box (outputs under gpurun_out/):
#   the GPU test suite, the default bench line (N=1, C2, live PMC), the 8-rank C3 shape with the
#   C4 / C5 configs, the 2-process launcher rehearsal and the launcher's refusal on one GPU.
# TAG names the outputs (default r03).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_suite.txt 2>&1 || { tail -30 gpurun_out/${TAG}_suite.txt; exit 1; }
  tail -2 gpurun_out/${TAG}_suite.txt
fi
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 400 python3 bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
  > gpurun_out/${TAG}_c345_8.json 2> gpurun_out/${TAG}_c345_8.err || { tail -20 gpurun_out/${TAG}_c345_8.err; exit 1; }
MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --no-cpu --pmc off \
  > gpurun_out/${TAG}_spawn2.json 2> gpurun_out/${TAG}_spawn2.err || { tail -20 gpurun_out/${TAG}_spawn2.err; exit 1; }
timeout -k 10 120 python3 bench.py --gpus 2 > gpurun_out/${TAG}_refuse2.json 2> gpurun_out/${TAG}_refuse2.err
echo "refuse rc=$?" | tee gpurun_out/${TAG}_refuse2.rc
echo done
