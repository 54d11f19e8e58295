#!/bin/bash
# Round-level GPU record: smoke, bench (with the CPU leg), rocprofv3 kernel
# trace of the bench, PMC traffic passes (stamped with this build), shard
# probes of the headline frame and C4, the BASELINE configs' timings.
# usage (GPU box): bash tools/gpu_round2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 4 | tail -12
bash tools/profile_traffic.sh $TAG > gpurun_out/traffic_$TAG.log 2>&1 || { tail -5 gpurun_out/traffic_$TAG.log; exit 1; }
tail -1 gpurun_out/traffic_$TAG.log | cut -c1-200
timeout -k 10 300 python tools/shard_probe.py 1 2 4 8 > gpurun_out/shards_$TAG.jsonl || exit 1
timeout -k 10 300 python tools/shard_probe.py --flags "-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05" 1 2 4 8 >> gpurun_out/shards_$TAG.jsonl || exit 1
cat gpurun_out/shards_$TAG.jsonl
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || { tail -3 gpurun_out/configs_$TAG.err; exit 1; }
cat gpurun_out/configs_$TAG.jsonl | cut -c1-200
