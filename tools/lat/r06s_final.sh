# r06s: the GPU suite, smoke and the driver-form bench line on the final sources (after the ring
# fallback's direct form)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
STEPS="suite" TAG=r06s bash tools/gpu_session.sh &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06s_smoke.txt 2>&1 && tail -1 $O/r06s_smoke.txt &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/r06s_bench_k20.json 2> $O/r06s_bench_k20.err
