#!/bin/bash
# Per-iteration closest-hit launch time, query counts and step maxima
# (RTX_DEBUG=2, stats pass) of the 8-way shard 6 and the full frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-it2}
RTX_DEBUG=2 timeout -k 10 100 python tools/tail_probe.py 8 6 > gpurun_out/it8_$TAG.txt 2>&1 || exit 1
RTX_DEBUG=2 timeout -k 10 100 python tools/tail_probe.py 1 0 > gpurun_out/it1_$TAG.txt 2>&1 || exit 1
grep "closest-hit launch" gpurun_out/it8_$TAG.txt | head -24
grep "closest-hit launch" gpurun_out/it1_$TAG.txt | head -24
