# r06i: the whole GPU suite, smoke, the default bench line (C2 through the all-pairs XML tiers) and
# the 8-process one-GPU rehearsal with the tuning keys on one collective stream per process
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/r06i_suite.txt 2>&1 && tail -2 $O/r06i_suite.txt &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06i_smoke.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/r06i_bench.json 2> $O/r06i_bench.err &&
MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 8 --steps 20 --warmup 5 \
  > $O/r06i_rehearse_8.json 2> $O/r06i_rehearse_8.err
