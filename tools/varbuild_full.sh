#!/bin/bash
# A measurement variant with whole per-type kernel objects rebuilt with extra flags, linked with the
# main build's other objects (brought up to date first; the layout guard of tools/varbuild.sh).
#   bash tools/varbuild_full.sh tools/lat/libvar_x.so "i8 f32 bf16" -DSOME_VARIANT
set -e
OUT=$1; TYPES=$2; shift 2
B=build/obj_var_$(basename $OUT .so)
mkdir -p $B tools/lat
make -s -C msccl_amd/csrc -j8
pids=()
for t in $TYPES; do
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -Wall -Wno-unused-parameter -Wno-unused-variable -Wno-unused-result \
    -Imsccl_amd/csrc -Iinclude --offload-arch=gfx950 -munsafe-fp-atomics -Wshadow -ffp-contract=off "$@" \
    -Rpass-analysis=kernel-resource-usage -c msccl_amd/csrc/device/kernels_$t.hip -o $B/kernels_$t.o 2> $B/res_$t.txt &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
OBJS=$(ls build/obj/*.o build/obj/device/*.o)
for t in $TYPES; do OBJS=$(echo "$OBJS" | grep -v "kernels_$t.o"); done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--no-undefined -o $OUT $OBJS $B/kernels_*.o -lpthread
python3 tools/check_layout.py $OUT || { rm -f $OUT; exit 1; }
echo built $OUT
