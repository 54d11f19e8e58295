#!/bin/bash
# GPU record of the current tree (run on the GPU box through gpurun), in the
# order given; every step has its own time limit and the first failure ends
# the script.
#   parity   pytest -m gpu (the whole GPU suite)
#   smoke    __graft_entry__.smoke()
#   bench    bench.py with the CPU leg and the parity block
#   prof     rocprofv3 --kernel-trace --stats of the bench (3 frames + warmup)
#   pmc      tools/profile_traffic.sh (FETCH / WRITE / TCC / SQ / VALU-mix
#            passes, stamped with this build), then the bench again so its
#            line carries this build's traffic and VALU fractions, and
#            tools/kernel_roofline.py (per-kernel roofline; needs prof)
#   shards   tools/shard_probe.py: headline, C4, R1 and C5 at 1 and 8 shards
#   configs  tools/bench_configs.py (BASELINE C1-C5)
# usage: bash tools/gpu_record.sh TAG step...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    parity)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
      tail -1 gpurun_out/pytest_$TAG.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
      tail -1 gpurun_out/smoke_$TAG.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
        || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
      tail -1 gpurun_out/bench_$TAG.json | cut -c1-400 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp)
      export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
        -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1 \
        || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
      python3 tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 10 | tail -6 ;;
    pmc)
      export TMPDIR=/tmp
      bash tools/profile_traffic.sh $TAG > gpurun_out/traffic_$TAG.log 2>&1 || { tail -5 gpurun_out/traffic_$TAG.log; exit 1; }
      tail -1 gpurun_out/traffic_$TAG.log | cut -c1-300
      timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench2_$TAG.json \
        2> gpurun_out/bench2_$TAG.err || { tail -5 gpurun_out/bench2_$TAG.err; exit 1; }
      tail -1 gpurun_out/bench2_$TAG.json | cut -c1-300
      if [ -f gpurun_out/prof_$TAG/run_kernel_stats.csv ]; then
        python3 tools/kernel_roofline.py gpurun_out/bench2_$TAG.json gpurun_out/prof_$TAG/run_kernel_stats.csv 10 \
          profiles/traffic_$TAG.json > gpurun_out/kernel_roofline_$TAG.json || exit 1
      fi ;;
    shards)
      : > gpurun_out/shards_$TAG.jsonl
      for fl in "-w 1920 -r 5 -O r -A 4" "-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05"; do
        timeout -k 10 300 python tools/shard_probe.py --flags "$fl" 1 8 >> gpurun_out/shards_$TAG.jsonl || exit 1
      done
      timeout -k 10 300 python tools/shard_probe.py --scene trimesh2_glass.ray --flags "-w 1920 -r 5 -O r -A 4" 1 8 \
        >> gpurun_out/shards_$TAG.jsonl || exit 1
      timeout -k 10 400 python tools/shard_probe.py --scene dragon.ray --flags "-w 3840 -r 5 -O a -A 8" 1 8 \
        >> gpurun_out/shards_$TAG.jsonl || exit 1
      cat gpurun_out/shards_$TAG.jsonl ;;
    configs)
      timeout -k 10 400 python tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err \
        || { tail -3 gpurun_out/configs_$TAG.err; exit 1; }
      cut -c1-200 gpurun_out/configs_$TAG.jsonl ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
