#!/bin/bash
# tail-switch iteration A/B on the full headline frame and its 8-way shards
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for e in "RTX_TAIL_ITER=0" "RTX_TAIL_ITER=1" "RTX_TAIL_ITER=2" "RTX_TAIL_ITER=3" "RTX_TAIL_ITER=5"; do
  env $e timeout -k 10 200 python tools/shard_probe.py 1 8 | sed "s|^|[$e] |" || exit 1
done
