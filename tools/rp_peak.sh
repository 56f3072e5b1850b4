#!/bin/bash
# Pre-register-allocation VGPR pressure of one resident-kernel shape (llc's amdgpu-print-rp on the MIR after
# the machine scheduler): tools/rp_peak.sh SRC.hip "X(250,250)" [extra hipcc flags...].  Prints the peak and
# the live-in registers of the peak block by defining opcode.  Measurement tool only.
set -e
SRC=$1; SH=$2; shift 2
L=/opt/rocm/lib/llvm/bin
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Xclang -target-feature -Xclang -packed-fp32-ops --cuda-device-only \
  -emit-llvm -c -o /tmp/rp.bc "$SRC" "-DRS_SHAPES_OVERRIDE(X)=$SH" "$@" 2>/dev/null
$L/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -mattr=-packed-fp32-ops -O3 -stop-after=machine-scheduler /tmp/rp.bc -o /tmp/rp.mir
$L/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -run-pass=amdgpu-print-rp /tmp/rp.mir -o /dev/null > /tmp/rp.txt 2>&1
python3 - <<'PY'
import re, collections
L=open('/tmp/rp.txt').read().splitlines()
best=(0,0,None); blk=None; blkline={}
for i,l in enumerate(L):
    m=re.match(r'\s*(bb\.\d+)',l)
    if m: blk=m.group(1); blkline[blk]=i
    m=re.match(r'\s+(\d+)\s+(\d+)\s+(\S.*)$',l)
    if m and int(m.group(2))>best[0]: best=(int(m.group(2)),i,blk)
print('peak VGPR', best[0], 'in', best[2], L[best[1]].strip()[:150])
j=blkline[best[2]]+1
while 'Live-in' not in L[j]: j+=1
live=re.findall(r'%(\d+):([0-9A-F]+)',L[j])
M=open('/tmp/rp.mir').read().splitlines()
defs={}
for l in M:
    m=re.match(r'\s+(?:early-clobber\s+|undef\s+)?%(\d+)(?:\.\w+)?:(\w+)\s*=\s*(?:(?:contract|nofpexcept|nsz|afn|reassoc|nuw|nsw|disjoint)\s+)*(\S+)',l)
    if m and m.group(1) not in defs: defs[m.group(1)]=(m.group(2),m.group(3))
cat=collections.Counter()
for v,mask in live:
    cls,op=defs.get(v,('?','?'))
    if 'vgpr' in cls or 'vreg' in cls or 'av_' in cls:
        cat[(cls,op)]+=max(1,bin(int(mask,16)).count('1')//2)
for k,c in cat.most_common(12): print(' ',c,k)
PY
