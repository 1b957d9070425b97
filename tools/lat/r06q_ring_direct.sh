# r06q: the ring fallback's Simple ReduceScatter / AllGather, 8 co-resident ranks, 8 MiB per rank
# block, graph replay: the direct form against the ring's FIFOs (MSCCL_AMD_DIRECT=0), two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for r in 1 2; do
  for c in rs ag; do
    for d in 1 0; do
      x=$(MSCCL_AMD_DIRECT=$d timeout -k 5 120 python tools/lat_one.py --schedule fbring --coll $c --bytes 8388608 --ranks 8 \
          --dtype 7 --graph --iters 40 2>&1 | grep -v amdgpu.ids) || exit 1
      echo "DIRECT=$d $c: $x" | tee -a $O/r06q_ring_direct.txt
    done
  done
done
