#!/bin/bash
# A/B of library variants over the headline (1 and 8 shards), R1, C4 and C5
# (tools/shard_probe.py, same box).  Each argument is one configuration:
# env assignments separated by ','; "lib=NAME" selects
# lib/variants/librtx_hip_NAME.so (tools/build_variants.sh); "" = default.
# AB_C5=1 adds the 1M-face dragon (C5, 8x8 adaptive at 3840x2160, 1 shard).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "$@"; do
  envs=""
  for a in $(echo "$cfg" | tr ',' ' '); do
    case $a in
      lib=*) envs="$envs RTX_HIP_LIB=$GRAFT_REPO_ROOT/cs378hgraphics-raytracer_amd/lib/variants/librtx_hip_${a#lib=}.so" ;;
      *) envs="$envs $a" ;;
    esac
  done
  env $envs timeout -k 10 200 python tools/shard_probe.py 1 8 | sed "s|^|[$cfg] |" || exit 1
  env $envs timeout -k 10 200 python tools/shard_probe.py --scene trimesh2_glass.ray 1 | sed "s|^|[$cfg] |" || exit 1
  env $envs timeout -k 10 200 python tools/shard_probe.py --flags "-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05" 1 8 | sed "s|^|[$cfg] |" || exit 1
  if [ -n "$AB_C5" ]; then
    env $envs timeout -k 10 300 python tools/shard_probe.py --scene dragon.ray --flags "-w 3840 -r 5 -O a -A 8" 1 | sed "s|^|[$cfg] |" || exit 1
  fi
done
