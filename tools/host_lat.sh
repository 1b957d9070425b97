#!/bin/bash
# host_lat variants + a kernel-trace profile of the small AllReduce (GPU box).
#   tools/host_lat.sh [schedule: pair|fallback]
set -e
mkdir -p gpurun_out/hl
o=gpurun_out/hl/host.txt
: > $o
if [ "${1:-pair}" = pair ]; then
  python -c "from msccl_amd import xmlgen; open('/tmp/hl_pair.xml','w').write(xmlgen.allreduce_pair_oneshot(1, 'LL'))"
  export MSCCL_XML_FILES=/tmp/hl_pair.xml
fi
for args in "2 128 2000 0 0" "2 128 2000 1 0" "2 4096 2000 0 0"; do
  echo "## $args" >> $o
  timeout -k 10 60 ./tools/host_lat $args >> $o 2>&1
  MSCCL_AMD_SMALL_KERNEL=0 timeout -k 10 60 ./tools/host_lat $args >> $o 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/hl/prof -o run -- $GRAFT_REPO_ROOT/tools/host_lat 2 128 2000 0 0 > $GRAFT_REPO_ROOT/gpurun_out/hl/prof.log 2>&1
