#!/bin/bash
# Per-iteration query counts (RTX_DEBUG=2) of the full headline frame and of
# its 8-way shard 6, plus the kernel timeline of one full frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-it}
RTX_DEBUG=2 timeout -k 10 100 python tools/tail_probe.py 8 6 > gpurun_out/it8_$TAG.txt 2>&1 || exit 1
RTX_DEBUG=2 timeout -k 10 100 python tools/tail_probe.py 1 0 > gpurun_out/it1_$TAG.txt 2>&1 || exit 1
grep "rtx group 0 " gpurun_out/it8_$TAG.txt | head -20
grep "rtx group 0 " gpurun_out/it1_$TAG.txt | head -20
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl1_$TAG -o run -- python3 tools/shard_probe.py 1 > gpurun_out/tl1_$TAG.log 2>&1 || exit 1
f=$(ls gpurun_out/tl1_$TAG/*/run_kernel_trace.csv gpurun_out/tl1_$TAG/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/timeline.py $f 3 > gpurun_out/tl1_${TAG}_frame.txt
head -60 gpurun_out/tl1_${TAG}_frame.txt
