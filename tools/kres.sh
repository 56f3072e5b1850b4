#!/bin/bash
# kernel resources (scratch, VGPRs, spills) of a built object: tools/kres.sh <obj.o> [name-filter]
B=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
$B/llvm-objcopy --dump-section .hip_fatbin=$d/fb.bin "$1" $d/x.o || exit 1
T=$($B/clang-offload-bundler --list --type=o --input=$d/fb.bin | grep gfx950)
$B/clang-offload-bundler --unbundle --type=o --targets=$T --input=$d/fb.bin --output=$d/k.co || exit 1
$B/llvm-readelf --notes $d/k.co | python3 -c "
import sys, re
f = sys.argv[1] if len(sys.argv) > 1 else ''
for blk in sys.stdin.read().split('.name:')[1:]:
    name = blk.split()[0]
    if f not in name: continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', blk) or [0, '?'])[1]
    print(f'{name[:64]:64s} scratch {g(\"private_segment_fixed_size\"):>4s} vgpr {g(\"vgpr_count\"):>3s} spill {g(\"vgpr_spill_count\")}')
" "$2"
rm -rf $d
