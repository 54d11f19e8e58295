# Ray-tree forking check on the GPU box: parity suite (every render path,
# forking included), then the shard probe with and without forking.
# usage: bash tools/fork_probe.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-fork}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo pytest_rc=$rc; tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/shard_probe.py 1 2 4 8 > gpurun_out/shards_$TAG.jsonl 2>&1 || { tail -5 gpurun_out/shards_$TAG.jsonl; exit 1; }
cat gpurun_out/shards_$TAG.jsonl
RTX_FORK=0 timeout -k 10 300 python -u tools/shard_probe.py 4 8 > gpurun_out/shards_${TAG}_nofork.jsonl 2>&1 || { tail -5 gpurun_out/shards_${TAG}_nofork.jsonl; exit 1; }
cat gpurun_out/shards_${TAG}_nofork.jsonl
for d in 2 4; do
RTX_FORK_DEPTH=$d timeout -k 10 300 python -u tools/shard_probe.py 8 > gpurun_out/shards_${TAG}_d$d.jsonl 2>&1 || { tail -5 gpurun_out/shards_${TAG}_d$d.jsonl; exit 1; }
echo depth $d; cat gpurun_out/shards_${TAG}_d$d.jsonl
done
