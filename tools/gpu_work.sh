#!/bin/bash
# Traversal work counts (bench.py's stats pass) for the default library and
# the variants named as arguments
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "" "$@"; do
  if [ -n "$v" ]; then L="RTX_HIP_LIB=$GRAFT_REPO_ROOT/cs378hgraphics-raytracer_amd/lib/variants/librtx_hip_$v.so"; else L="X=1"; fi
  env $L timeout -k 10 200 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/work_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/work_$v.json'));print('[$v]',d['ms_per_step'],d['work'])"
done
