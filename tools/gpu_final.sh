#!/bin/bash
# End-of-session GPU record: parity suite, then tools/gpu_round2.sh (smoke,
# bench with the CPU leg, rocprof kernel stats, PMC traffic, shard probes,
# configs), then the bench once more so its line carries the PMC traffic of
# this very build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_round2.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || exit 1
tail -1 gpurun_out/bench2_$TAG.json | cut -c1-600
