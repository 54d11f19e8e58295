#!/bin/bash
# Print per-kernel VGPR/AGPR/scratch/occupancy of the HIP library source.
cd "$(dirname "$0")/../cs378hgraphics-raytracer_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I../include \
  "$@" -c csrc/hip/rtx_render.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | \
  python3 -c "
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); print(); print(cur[:70], end=' '); continue
    for k in ('VGPRs:','AGPRs:','ScratchSize \[bytes/lane\]:','Occupancy \[waves/SIMD\]:'):
        m=re.search(k+r' (\d+)',l)
        if m: print(k.split()[0]+m.group(1), end=' ')
print()"
