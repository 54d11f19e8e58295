#!/bin/bash
# re-entry check of the rebuilt tree: parity suite, short bench, tail-switch
# iteration A/B on the full frame and its 8-way shards
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02p}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-400 gpurun_out/bench_$TAG.json
bash tools/gpu_tailit.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$TAG -o run -- python3 tools/shard_probe.py 8 > gpurun_out/tl_$TAG.log 2>&1 || exit 1
f=$(ls gpurun_out/tl_$TAG/*/run_kernel_trace.csv gpurun_out/tl_$TAG/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/timeline.py $f 3 --brief
python3 tools/timeline.py $f 3 > gpurun_out/tl_${TAG}_frame.txt
