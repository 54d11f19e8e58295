#!/bin/bash
# A/B of environment settings on the headline bench (one line per setting).
# usage: bash tools/gpu_ab_env.sh TAG "ENV1=.. ENV2=.." "ENV1=.." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || { tail -3 gpurun_out/ab_${TAG}_$i.err; exit 1; }
  echo "[$e] $(python3 -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_$i.json'));print(d['ms_per_step'], d['value'])")"
done
