# r06d: the pipelined two-phase fold: GPU parity of the lowered large calls, then the C3 sweep and
# the 2-rank headline with their secondary schedule lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_twophase.py > $O/r06d_twophase.txt 2>&1 &&
timeout -k 10 240 python bench.py --vranks 8 --dtype fp16 --no-cpu --pmc off --steps 20 --warmup 5 > $O/r06d_c3.json 2> $O/r06d_c3.err &&
timeout -k 10 240 python bench.py --no-cpu --pmc off --steps 20 --warmup 5 --sizes 33554432 > $O/r06d_c2.json 2> $O/r06d_c2.err
