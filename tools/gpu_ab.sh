#!/bin/bash
# A/B of librtx_hip builds on the headline frame (run on the GPU box).
# usage: bash tools/gpu_ab.sh TAG [pytest] -- VAR=value ... (each arg after
# -- is one configuration: env assignments separated by ',', "" = default)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out
if [ "$1" = "pytest" ]; then
  shift
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
  echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || exit 1
fi
[ "$1" = "--" ] && shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --no-cpu --steps 5 > gpurun_out/ab_${TAG}_$i.log 2>&1 || { echo "FAIL [$cfg]"; tail -5 gpurun_out/ab_${TAG}_$i.log; exit 1; }
  echo "[$cfg] $(tail -1 gpurun_out/ab_${TAG}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s", d["ms_per_step"], "ms", "frac", d["roofline"]["frac"], "nodes/tris", d["roofline"]["algorithmic_bytes_per_launch"])')"
done
