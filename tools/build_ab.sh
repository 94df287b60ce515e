#!/bin/bash
# A/B variant of libskm: one source (SRC=build | annotate | matrix, default build) recompiled with
# extra defines, linked with the default objects of the others.
#   tools/build_ab.sh NAME -DX=Y ...  ->  signature_kmers_amd/libskm_NAME.so (load with SKM_LIB_PATH)
set -eu
NAME=$1; shift
SRC=${SRC:-build}
make -s -j8 signature_kmers_amd/libskm.so
mkdir -p build/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -DSKM_WITH_RCCL \
  -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Wall -Wno-unused-function "$@" \
  -c signature_kmers_amd/csrc/skm_$SRC.hip -o build/ab/skm_${SRC}_$NAME.o
OBJS=""
for s in build annotate matrix; do
  if [ $s = $SRC ]; then OBJS="$OBJS build/ab/skm_${SRC}_$NAME.o"; else OBJS="$OBJS build/obj/skm_$s.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o signature_kmers_amd/libskm_$NAME.so $OBJS \
  build/obj/skm_host.o build/obj/skm_bdz.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
