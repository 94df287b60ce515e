#!/bin/bash
# A/B variant of libskm: skm_build.hip recompiled with extra defines, linked with the default
# objects.  tools/build_ab.sh NAME -DX=Y ...  ->  signature_kmers_amd/libskm_NAME.so (SKM_LIB_PATH)
set -eu
NAME=$1; shift
make -s -j8 signature_kmers_amd/libskm.so
mkdir -p build/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -DSKM_WITH_RCCL \
  -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Wall -Wno-unused-function "$@" \
  -c signature_kmers_amd/csrc/skm_build.hip -o build/ab/skm_build_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o signature_kmers_amd/libskm_$NAME.so build/ab/skm_build_$NAME.o \
  build/obj/skm_annotate.o build/obj/skm_matrix.o build/obj/skm_host.o build/obj/skm_bdz.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
