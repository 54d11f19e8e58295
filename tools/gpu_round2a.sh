#!/bin/bash
# round-2 GPU check: parity suite + a short bench (no CPU leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r02a_pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
rc=$?
cat gpurun_out/r02a_bench.json
exit $rc
