#!/bin/bash
# round-2 check: parity suite, then A/B of tail switch / trace-grid split /
# fork depth on the headline frame, and the debug counters of one frame
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02m}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh $TAG RTX_TAIL=1000000 RTX_TAIL=4000000 RTX_TAIL=12000000 RTX_TGRID_DIV=2 RTX_TGRID_DIV=3 RTX_FORK_DEPTH=4 || exit 1
RTX_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/dbg_$TAG.json 2> gpurun_out/dbg_$TAG.err || exit 1
grep "rtx trace\|rtx tail" gpurun_out/dbg_$TAG.err | head -5
