# r06j: the 2-process C2 tier tests, smoke, the default bench line (C2 through the all-pairs XML
# tiers) and the 8-process one-GPU rehearsal with the tuning keys on one collective stream per process
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_lowering.py -m gpu -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/r06j_tests.txt 2>&1 && tail -2 $O/r06j_tests.txt &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06j_smoke.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/r06j_bench.json 2> $O/r06j_bench.err &&
MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 8 --steps 20 --warmup 5 \
  > $O/r06j_rehearse_8.json 2> $O/r06j_rehearse_8.err
