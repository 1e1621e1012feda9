#!/bin/bash
# Kernel resource metadata (VGPRs, scratch, LDS) from a built object, without a -S rebuild:
# unbundle the gfx950 code object and read its AMDGPU metadata notes.
# Usage: tools/kmeta.sh [obj] [kernel-name regex]
OBJ=${1:-torch-admm-deconv_amd/csrc/build/admm_capi.o}
PAT=${2:-.}
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin="$T/fb.bin" "$OBJ" "$T/null.o" || exit 1
$B/clang-offload-bundler -type=o -targets=hipv4-amdgcn-amd-amdhsa--gfx950 -input="$T/fb.bin" -output="$T/k.hsaco" -unbundle || exit 1
$B/llvm-readelf --notes "$T/k.hsaco" | python3 -c "
import sys, re, subprocess
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split('  - .agpr_count')[1:]:
    def g(k):
        m = re.search(r'\.' + k + r':\s+(\S+)', blk)
        return m.group(1) if m else '?'
    name = subprocess.run(['c++filt', g('name')], capture_output=True, text=True).stdout.strip()
    name = re.sub(r'\(.*', '', name).replace('admm::', '').replace('(anonymous namespace)::', '')
    if pat.search(name):
        print(f\"{name[:70]:70s} vgpr={g('vgpr_count')} sgpr={g('sgpr_count')} scratch={g('private_segment_fixed_size')} lds={g('group_segment_fixed_size')}\")
" "$PAT"
rm -rf "$T"
