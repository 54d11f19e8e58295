#!/bin/bash
# Kernel-trace profile of the bench command (run on the GPU box).
# usage: tools/profile_run.sh TAG [bench args...]
set -e
TAG=$1; shift
mkdir -p gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu "$@"
