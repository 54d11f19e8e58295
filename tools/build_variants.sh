#!/bin/bash
# Build tuning variants of librtx_hip.so into cs378hgraphics-raytracer_amd/lib/variants/
# usage: tools/build_variants.sh NAME "-DFLAG=.. ..." [NAME "FLAGS"]...
cd "$(dirname "$0")/../cs378hgraphics-raytracer_amd"
mkdir -p lib/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-gpu-rdc \
    -munsafe-fp-atomics -Wno-unused-function -Wno-unused-variable -I../include $flags -shared \
    -o lib/variants/librtx_hip_$name.so csrc/hip/rtx_render.hip &
done
wait
ls -la lib/variants
