#!/bin/bash
# A/B of RTX_LEAF_K on the full headline frame and the 8-way shards
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_leafk.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_leafk.log
[ $rc -ne 0 ] && exit $rc
for k in 65 4 16 32 48; do
  RTX_LEAF_K=$k timeout -k 10 200 python tools/shard_probe.py 1 8 | sed "s|^|[K=$k] |" || exit 1
done
