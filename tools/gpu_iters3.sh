#!/bin/bash
# Per-iteration closest-hit and walk launch times (RTX_DEBUG=2, stats pass,
# synchronous) of the full frame; optional variant library name $1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "$1" ] && export RTX_HIP_LIB=$GRAFT_REPO_ROOT/cs378hgraphics-raytracer_amd/lib/variants/librtx_hip_$1.so
RTX_DEBUG=2 timeout -k 10 100 python tools/tail_probe.py 1 0 > gpurun_out/it1_cur.txt 2>&1 || exit 1
grep "iter [0-2]:" gpurun_out/it1_cur.txt | grep "group 0" | head -18
grep "trace steps per query" gpurun_out/it1_cur.txt
