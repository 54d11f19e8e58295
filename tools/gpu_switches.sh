#!/bin/bash
# Parity of the documented switches: the advance-launch first iteration
# (RTX_CAM_FIRST=0) and no postponing (RTX_LEAF_K=65) on the GPU parity suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RTX_CAM_FIRST=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_camfirst0.log 2>&1 || { tail -5 gpurun_out/pytest_camfirst0.log; exit 1; }
tail -1 gpurun_out/pytest_camfirst0.log
RTX_LEAF_K=65 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_leafk65.log 2>&1 || { tail -5 gpurun_out/pytest_leafk65.log; exit 1; }
tail -1 gpurun_out/pytest_leafk65.log
