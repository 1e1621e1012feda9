#!/bin/bash
# quick resource check of explicitly instantiated kernels (build_kt/inst.hip) against the tree's headers
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Itorch-admm-deconv_amd/csrc -ffp-contract=off -fno-slp-vectorize $KT_FLAGS -c build_kt/inst.hip -o build_kt/inst.o 2>&1 | grep -E "error" -A3 | head -20
tools/kmeta.sh build_kt/inst.o "${1:-k_pass}"
