#!/bin/bash
# The GPU suite under the library's alternative modes (GPU box): the
# sequential machine (RTX_FUSE=0), two frame contexts (RTX_CONTEXTS=2), no
# frame pipelining (RTX_PIPELINE=0), no ray-tree forks (RTX_FORK=0).  Every
# mode must give the same images (the parity tests compare against the CPU
# restatement; bit-exact rgb8 outside rounding boundaries).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "gpurun_out/robust_${cfg//[= ]/_}.log" 2>&1 || { echo "[$cfg] FAIL"; tail -20 "gpurun_out/robust_${cfg//[= ]/_}.log"; exit 1; }
  echo "[$cfg] $(tail -1 "gpurun_out/robust_${cfg//[= ]/_}.log")"
done
