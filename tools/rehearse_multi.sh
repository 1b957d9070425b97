#!/bin/bash
# Rehearse bench.py's multi-process path (one rank per process, hipIpc FIFOs) on a one-GPU box:
# every rank on cuda:0.  The driver runs the real N-GPU case; this only checks the plumbing.
set -o pipefail
export MSCCL_AMD_BENCH_ONE_GPU=1
for n in ${NS:-2 4}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 --extras ${EXTRAS:-C4,C5} \
    > gpurun_out/multi_$n.json 2> gpurun_out/multi_$n.err || { tail -30 gpurun_out/multi_$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/multi_$n.json')); print($n, d['value'], d['dtype'], d['config']['workload'], d.get('configs'))" || exit 1
done
