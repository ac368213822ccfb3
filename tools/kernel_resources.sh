#!/bin/bash
# usage: res.sh file.hip  -> per-kernel vgpr/sgpr/spill/occupancy
f=$1; b=$(basename $f .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I/root/repo/include -I. -c $f --save-temps=obj -o /tmp/$b.o -Rpass-analysis=kernel-resource-usage 2> /tmp/$b-usage.txt
grep error /tmp/$b-usage.txt | head -5
python3 - "$b" <<'PY'
import re,sys
txt=open(f'/tmp/{sys.argv[1]}-usage.txt').read()
for blk in re.split(r'Function Name: ',txt)[1:]:
    name=blk.split()[0]
    g=lambda k: re.search(k+r': (\d+)',blk).group(1)
    print(name[:44], 'vgpr',g('VGPRs'),'sgpr',g('SGPRs'),'scratch',g(r'ScratchSize \[bytes/lane\]'),'occ',g(r'Occupancy \[waves/SIMD\]'),'lds',g(r'LDS Size \[bytes/block\]'))
PY
