# r06f: the direct form of Simple schedules: GPU parity, then C4 / C5 on 8 co-resident ranks with
# and without it (MSCCL_AMD_DIRECT), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_direct.py > $O/r06f_direct_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu --pmc off --no-secondary \
  --steps 10 --warmup 3 > $O/r06f_c45_direct.json 2> $O/r06f_c45_direct.err &&
MSCCL_AMD_DIRECT=0 timeout -k 10 300 python bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu \
  --pmc off --no-secondary --steps 10 --warmup 3 > $O/r06f_c45_fifo.json 2> $O/r06f_c45_fifo.err
