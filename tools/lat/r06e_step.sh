# r06e: two-phase fold packs per FIFO step (MSCCL_AMD_TWO_PHASE_STEP) 2048 / 1024 / 512 / 256,
# alternating twice on one box: C3 shape (8 co-resident ranks, fp16) 1-32 MiB and RCCL's 8n-32tb
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for rep in 1 2; do
  for st in 2048 1024 512 256; do
    MSCCL_AMD_TWO_PHASE_STEP=$st timeout -k 10 200 python bench.py --vranks 8 --dtype fp16 --no-cpu --pmc off \
      --steps 20 --warmup 5 --sizes 1048576,4194304,16777216,33554432 > $O/r06e_st${st}_$rep.json 2> $O/r06e_st${st}_$rep.err || exit 1
  done
done
