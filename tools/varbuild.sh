#!/bin/bash
# A measurement variant of the fp32 kernels: kernels_f32.hip compiled with extra flags (and only the
# small-call and fold kernels, MSCCL_SMALL_ONLY), linked with the main build's other objects.
#   bash tools/varbuild.sh tools/lat/libvar_a.so -DSOME_VARIANT
# Run from the repo root (the other objects come from build/obj, brought up to date first).
# Guard (round 6, the r05k fault): a -D flag that changes RankWork (devcomm.h) reaches only this
# object, and build/obj may hold host objects older than the headers; either way the variant's
# kernels and the host disagree on the launch-argument layout.  `make` first, then the host-only
# layout check on the linked library (tools/check_layout.py): a split fails here, before any GPU run.
set -e
OUT=$1; shift
B=build/obj_var_$(basename $OUT .so)
mkdir -p $B tools/lat
make -s -C msccl_amd/csrc -j8
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -Wall -Wno-unused-parameter -Wno-unused-variable -Wno-unused-result \
  -Imsccl_amd/csrc -Iinclude --offload-arch=gfx950 -munsafe-fp-atomics -Wshadow -ffp-contract=off \
  -DMSCCL_SMALL_ONLY "$@" -Rpass-analysis=kernel-resource-usage -c msccl_amd/csrc/device/kernels_f32.hip -o $B/kernels_f32.o 2> $B/res.txt || { cat $B/res.txt; exit 1; }
OBJS=$(ls build/obj/*.o build/obj/device/*.o | grep -v kernels_f32.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--no-undefined -o $OUT $OBJS $B/kernels_f32.o -lpthread
python3 tools/check_layout.py $OUT || { rm -f $OUT; exit 1; }
echo built $OUT
