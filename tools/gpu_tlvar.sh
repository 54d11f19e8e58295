#!/bin/bash
# Kernel timeline of one full headline frame for a variant library and env
# usage: bash tools/gpu_tlvar.sh TAG LIBNAME|- [VAR=value ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; LIBN=$2; shift 2
[ "$LIBN" != "-" ] && export RTX_HIP_LIB=$GRAFT_REPO_ROOT/cs378hgraphics-raytracer_amd/lib/variants/librtx_hip_$LIBN.so
for a in "$@"; do export "$a"; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlv_$TAG -o run -- python3 tools/shard_probe.py 1 > gpurun_out/tlv_$TAG.log 2>&1 || exit 1
grep max_ms gpurun_out/tlv_$TAG.log
f=$(ls gpurun_out/tlv_$TAG/*/run_kernel_trace.csv gpurun_out/tlv_$TAG/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/timeline.py $f 3 > gpurun_out/tlv_${TAG}_frame.txt
head -30 gpurun_out/tlv_${TAG}_frame.txt
tail -7 gpurun_out/tlv_${TAG}_frame.txt
