#!/bin/bash
# The GPU suite under the library's alternative modes (GPU box): the
# sequential machine (RTX_FUSE=0), two frame contexts (RTX_CONTEXTS=2), no
# frame pipelining (RTX_PIPELINE=0), no ray-tree forks (RTX_FORK=0), short
# walk stacks with overflow columns on every frame (RTX_TEST_LDS_STACK=2),
# and the bounds-check build (RTX_HIP_LIB=.../lib/variants/librtx_hip_chk.so,
# tools/build_variants.sh chk -DRTX_BOUNDS_CHECK).  Every mode must give the
# same images (the parity tests compare against the CPU restatement;
# bit-exact rgb8 outside rounding boundaries).
# usage: bash tools/robust_suite.sh "RTX_FUSE=0" "RTX_TEST_LDS_STACK=2" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "$@"; do
  log="gpurun_out/robust_$(basename "${cfg//[= ]/_}").log"
  env $cfg timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$log" 2>&1 || { echo "[$cfg] FAIL"; tail -20 "$log"; exit 1; }
  echo "[$cfg] $(tail -1 "$log")"
done
