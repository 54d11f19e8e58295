#!/bin/bash
# shard-8 timing (tools/shard_probe.py 8) for each librtx_hip build given
# (paths relative to the repo; "" = the default build).  GPU box only.
cd $GRAFT_REPO_ROOT
for lib in "$@"; do
  RTX_HIP_LIB=$lib timeout -k 10 300 python tools/shard_probe.py 1 8 | sed "s|^|[${lib:-default}] |" || exit 1
done
