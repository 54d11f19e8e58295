#!/bin/bash
# fused-walk check: parity suite, then the headline frame with and without fused walks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-fuse}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
for f in 1 0 1; do
  RTX_FUSE=$f timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_${TAG}_f$f.json 2> gpurun_out/bench_${TAG}_f$f.err || exit 1
  echo "RTX_FUSE=$f $(python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_f$f.json'));print(d['ms_per_step'], d['value'])")"
done
