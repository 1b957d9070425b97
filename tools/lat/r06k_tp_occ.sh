# r06k (FAULTED: its variant set G = 4 against the 16-line ldLines16; see profiles/r06k_tp_occ.txt; the
# variant cannot be built any more): the two-phase fold built for two workgroups per CU (tools/lat/libvar_tp2.so: -DMSCCL_TP_OCC=2
# -DMSCCL_TP_G=4, 116 VGPRs) against the main build (one per CU, 166 VGPRs), C3 32 MiB on 8
# co-resident ranks, alternating: main, variant at 32 workgroups per rank (TARGET_WGS 256),
# variant at 64 (TARGET_WGS 512), three rounds; plus RCCL's 8n-32tb file through the secondary line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
one() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  env MSCCL_AMD_LIB=$lib "$@" timeout -k 10 200 python bench.py --vranks 8 --dtype fp16 --sizes 33554432 --no-cpu \
    --pmc off --no-secondary --steps 20 --warmup 5 > $O/r06k_c3.json 2>> $O/r06k_c3.err || return 1
  python -c "
import json; d = json.load(open('$O/r06k_c3.json')); s = d['sweep'][-1]
print('$tag', s['kernel_ms'], s['busbw'], s['kernel'], d['verified'])" | tee -a $O/r06k_tp_occ.txt
}
for r in 1 2 3; do
  one main msccl_amd/libmsccl_amd.so &&
  one tp2_w256 tools/lat/libvar_tp2.so &&
  one tp2_w512 tools/lat/libvar_tp2.so MSCCL_AMD_TARGET_WGS=512 || exit 1
done
