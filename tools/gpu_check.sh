#!/bin/bash
# GPU check of the current tree: parity suite, full-frame and 8-way shard
# times, kernel timeline of the 8-way shards (frame index $2, default 27:
# shard 6's last render), debug counters of shard 6.
# usage: bash tools/gpu_check.sh TAG [frame]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-chk}
FR=${2:-27}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/shard_probe.py 1 8 || exit 1
timeout -k 10 200 python tools/shard_probe.py --flags "-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05" 1 8 || exit 1
RTX_DEBUG=1 timeout -k 10 100 python tools/tail_probe.py 8 6 > gpurun_out/dbg_$TAG.txt 2>&1 || exit 1
grep -v "^rtx group" gpurun_out/dbg_$TAG.txt | tail -6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$TAG -o run -- python3 tools/shard_probe.py 8 > gpurun_out/tl_$TAG.log 2>&1 || exit 1
f=$(ls gpurun_out/tl_$TAG/*/run_kernel_trace.csv gpurun_out/tl_$TAG/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/timeline.py $f $FR --brief
python3 tools/timeline.py $f $FR > gpurun_out/tl_${TAG}_frame.txt
