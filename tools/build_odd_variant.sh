#!/bin/bash
# A/B variant of the library that differs only in the fused odd-length row pass (odd_capi.hip): the other
# objects are copied from the default build, so only odd_capi.o is recompiled with the extra flags.
# -> tools/_variants/NAME.so (same sources, so the build-hash check passes under ADMMTOR_LIB_OVERRIDE)
# usage: bash tools/build_odd_variant.sh NAME "-DADMM_ODD_NT=192 ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
C=torch-admm-deconv_amd/csrc
rm -rf $C/build_$NAME && mkdir -p $C/build_$NAME tools/_variants
cp -p $C/build/*.o $C/build/build_hash.cpp $C/build_$NAME/
rm -f $C/build_$NAME/odd_capi.o
make -C $C -j8 OBJDIR=build_$NAME OUT=../../tools/_variants/$NAME.so \
  CXXFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -I../../include -ffp-contract=off -fno-slp-vectorize $*" ../../tools/_variants/$NAME.so >/dev/null
echo built tools/_variants/$NAME.so
