#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02o.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_r02o.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_tailit.sh || exit 1
timeout -k 10 300 python tools/bench_configs.py C5 C4 | cut -c1-250
