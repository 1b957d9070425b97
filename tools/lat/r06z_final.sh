# r06z: final-source evidence. PART=1: the GPU suite and smoke; PART=2: the bench line in the
# driver's form (--steps 20 --warmup 5, live PMC) and the default form, rocprofv3 kernel trace +
# stats + FETCH_SIZE / WRITE_SIZE of the C2 headline and of the 8-rank C3 / C4 / C5 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
if [ "$PART" = 1 ]; then
  STEPS="suite" TAG=r06z bash tools/gpu_session.sh &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06z_smoke.txt 2>&1 && tail -1 $O/r06z_smoke.txt
else
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/r06z_bench_k20.json 2> $O/r06z_bench_k20.err &&
  STEPS="bench prof prof8" TAG=r06z bash tools/gpu_session.sh
fi
