# r06g: the direct kernel with 4 packs per lane and up to 1024 workgroups per GPU (GPU parity, then
# C4 / C5 on 8 co-resident ranks at MSCCL_AMD_DIRECT_WGS = 512 / 1024 / 2048); the C2 sweep through
# the msccl-tools two-phase all-pairs XML against the pair one-shot tiers (driver form: 20 / 5);
# the 8-process one-GPU rehearsal of bench.py --gpus 8 with its tuning keys
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_direct.py > $O/r06g_direct_tests.txt 2>&1 &&
for w in 512 1024 2048; do
  MSCCL_AMD_DIRECT_WGS=$w timeout -k 10 300 python bench.py --vranks 8 --dtype fp16 --sizes 33554432 --extras C4,C5 --no-cpu \
    --pmc off --no-secondary --steps 10 --warmup 3 > $O/r06g_c45_w$w.json 2> $O/r06g_c45_w$w.err || exit 1
done &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --pmc off > $O/r06g_c2_pair.json 2> $O/r06g_c2_pair.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --pmc off --tiers 0:4096:1:a,4096:1073741825:16:a \
  > $O/r06g_c2_allpairs.json 2> $O/r06g_c2_allpairs.err &&
MSCCL_AMD_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 8 --steps 20 --warmup 5 \
  > $O/r06g_rehearse_8.json 2> $O/r06g_rehearse_8.err
