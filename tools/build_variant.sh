#!/bin/bash
# Build an A/B variant of the library with extra compile flags into tools/_variants/NAME.so
# (same sources, so the build-hash check of admmtor._native still passes under ADMMTOR_LIB_OVERRIDE).
# usage: bash tools/build_variant.sh NAME "-DFLAG=1 ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p tools/_variants
make -C torch-admm-deconv_amd/csrc -j8 OBJDIR=build_$NAME OUT=../../tools/_variants/$NAME.so \
  CXXFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -I../../include -ffp-contract=off -fno-slp-vectorize -DADMM_AB_BUILD=1 $*" ../../tools/_variants/$NAME.so >/dev/null
echo built tools/_variants/$NAME.so
