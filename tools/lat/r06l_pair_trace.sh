# r06l: where a lowered 2-rank pair call's device time goes (the pair kernel's MSCCL_LAT_TRACE
# points, tools/lat/libvar_lat.so = the fp32 kernels built with -DMSCCL_LAT_TRACE), 8 KiB / 64 KiB /
# 512 KiB through the two-phase all-pairs XML x16 (bench.py's C2 tier), graph replay
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
for b in 8192 65536 524288; do
  echo "== allpairs x16 $b B" >> $O/r06l_pair_trace.txt
  LAT_TRACE_SCHEDULE=allpairs MSCCL_AMD_LIB=tools/lat/libvar_lat.so MSCCL_AMD_TRACE=2 timeout -k 5 120 \
    python tools/lat_trace.py $b 16 >> $O/r06l_pair_trace.txt 2>&1 || exit 1
done
