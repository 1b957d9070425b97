# r06n: the two-phase fold built for two workgroups per CU (tools/lat/libvar_tp2.so: the fp16
# kernels with -DMSCCL_TP_OCC=2: 4 peers per batch through ldLinesPeers<4>, <= 128 VGPRs) against
# the main build (one per CU), C3 32 MiB on 8 co-resident ranks, alternating: main, variant at 32
# workgroups per rank (TARGET_WGS 256), variant at 64 (TARGET_WGS 512), three rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
one() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  env MSCCL_AMD_LIB=$lib "$@" timeout -k 10 200 python bench.py --vranks 8 --dtype fp16 --sizes 33554432 --no-cpu \
    --pmc off --no-secondary --steps 20 --warmup 5 > $O/r06n_c3.json 2>> $O/r06n_c3.err || return 1
  python -c "
import json; d = json.load(open('$O/r06n_c3.json')); s = d['sweep'][-1]
print('$tag', s['kernel_ms'], s['busbw'], s['kernel'], d['verified'])" | tee -a $O/r06n_tp_occ.txt
}
timeout -k 10 300 env MSCCL_AMD_LIB=tools/lat/libvar_tp2.so python -u -m pytest -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_twophase.py -m gpu -k "eight_rank or rccl" > $O/r06n_tests.txt 2>&1 &&
tail -1 $O/r06n_tests.txt &&
timeout -k 10 300 env MSCCL_AMD_LIB=tools/lat/libvar_tp2.so MSCCL_AMD_TARGET_WGS=512 python -u -m pytest -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_twophase.py -m gpu -k "eight_rank or rccl" >> $O/r06n_tests.txt 2>&1 &&
tail -1 $O/r06n_tests.txt &&
c2() {  # tag env...: C2 32 MiB (the lowered pair: flat workgroups per rank follow MSCCL_AMD_TARGET_WGS)
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --sizes 33554432 --no-cpu --pmc off --no-secondary --steps 20 --warmup 5 \
    > $O/r06n_c2.json 2>> $O/r06n_c3.err || return 1
  python -c "
import json; d = json.load(open('$O/r06n_c2.json')); s = d['sweep'][-1]
print('$tag', s['kernel_ms'], s['busbw'], s['kernel'], d['verified'])" | tee -a $O/r06n_tp_occ.txt
}
for r in 1 2 3; do
  c2 c2_w256 MSCCL_AMD_TARGET_WGS=256 &&
  c2 c2_w512 MSCCL_AMD_TARGET_WGS=512 &&
  one main msccl_amd/libmsccl_amd.so &&
  one tp2_w256 tools/lat/libvar_tp2.so &&
  one tp2_w512 tools/lat/libvar_tp2.so MSCCL_AMD_TARGET_WGS=512 || exit 1
done
