# SQ counters of small launches (one pass, <= 8 SQ counters)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/latpmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_IFETCH SQ_WAVES --output-format csv -d gpurun_out/latpmc/a -o run -- python3 tools/lat_one.py --schedule pair --bytes 128 --iters 100 > gpurun_out/latpmc/a.log 2>&1 || exit 1
