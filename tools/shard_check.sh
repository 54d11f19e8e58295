# Parity suite + shard probe (N = 1, 2, 4, 8 on one GPU).
# usage: bash tools/shard_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-shard}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo pytest_rc=$rc; tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/shard_probe.py 1 2 4 8 2>/dev/null > gpurun_out/shards_$TAG.jsonl || { tail -5 gpurun_out/shards_$TAG.jsonl; exit 1; }
cat gpurun_out/shards_$TAG.jsonl
