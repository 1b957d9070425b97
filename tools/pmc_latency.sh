set -o pipefail
export TMPDIR=/tmp MSCCL_AMD_TIMEOUT_SEC=20
O=gpurun_out/pmc_lat
mkdir -p $O
timeout -s KILL 90 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
for c in 0 1 4; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/c$c -o run -- python3 tools/latency_probe.py --case $c --iters 50 > $O/c$c.txt 2>&1 || exit 1
done
