#!/bin/bash
# Register / spill / LDS summary of the gfx950 kernels in one object of the
# build: bash tools/kres.sh conv [name-filter]
set -eo pipefail
B=/opt/rocm/lib/llvm/bin
O=${1:?object stem}; F=${2:-.}
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$(dirname "$0")/../road-vision-system_amd/csrc/build/$O.o"
$B/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
$B/llvm-readelf --notes $T/co | python3 -c "
import sys,re
cur={}
rows=[]
for l in sys.stdin:
    l=l.strip()
    m=re.match(r'-?\s*\.(\w+):\s+(.*)',l)
    if not m: continue
    k,v=m.groups()
    if k=='agpr_count' and cur: pass
    cur[k]=v
    if k=='wavefront_size':
        rows.append(cur); cur={}
for r in rows:
    n=r.get('name','?')
    if not re.search(sys.argv[1], n): continue
    print('%4s v %3s a %3s s sspill %3s vspill %3s lds %6s  %s'%(r.get('vgpr_count'),r.get('agpr_count'),r.get('sgpr_count'),r.get('sgpr_spill_count'),r.get('vgpr_spill_count'),r.get('group_segment_fixed_size'),n[:150]))
" "$F"
rm -rf $T
