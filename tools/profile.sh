#!/bin/bash
# rocprofv3 evidence for bench.py's headline launch (run on the GPU box from the repo root):
#   pass 1: kernel trace + stats (per-kernel durations)
#   pass 2: FETCH_SIZE alone, pass 3: WRITE_SIZE alone (they do not fit one TCC pass on gfx950)
# Every pass profiles the same command: the C2 headline size only, so every mscclKernel dispatch in
# it is a headline launch.  tools/parse_prof.py turns the CSVs into profiles/<tag>_*.
set -o pipefail
TAG=${1:-r01}
shift
# --pmc off: under rocprofv3 the bench must not start its own profiler child (an exec from a process
# the outer profiler has initialised); --no-secondary: every interpreter dispatch is a headline launch
ARGS=${@:-"--no-cpu --quiet --sizes 33554432 --steps 20 --warmup 5 --pmc off --no-secondary"}
# counters per dispatch: eager launches (one dispatch per step, no graph in the profiled process)
ARGS="$ARGS --eager"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.json || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.json || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.json || exit 1
python3 tools/parse_prof.py $OUT $TAG && cp profiles/${TAG}_* $OUT/   # profiles/ is not copied back from a GPU box
