#!/bin/bash
# Full headline frame: time (shard_probe 1, twice) and kernel timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-tl1}
timeout -k 10 100 python tools/shard_probe.py 1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl1_$TAG -o run -- python3 tools/shard_probe.py 1 > gpurun_out/tl1_$TAG.log 2>&1 || exit 1
f=$(ls gpurun_out/tl1_$TAG/*/run_kernel_trace.csv gpurun_out/tl1_$TAG/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/timeline.py $f 3 > gpurun_out/tl1_${TAG}_frame.txt
head -50 gpurun_out/tl1_${TAG}_frame.txt
tail -8 gpurun_out/tl1_${TAG}_frame.txt
timeout -k 10 100 python tools/shard_probe.py 1 || exit 1
