#!/bin/bash
# Kernel-trace summary + HBM traffic (PMC FETCH_SIZE / WRITE_SIZE passes) of the
# headline bench on the GPU box.  usage: bash tools/gpu_prof.sh TAG [pmc]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-prof}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 4
if [ "$2" = "pmc" ]; then
  bash tools/profile_traffic.sh $TAG || exit 1
fi
