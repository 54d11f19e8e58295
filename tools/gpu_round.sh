# Round-level GPU check: parity (all render paths), smoke, bench (with CPU
# baseline) and a rocprofv3 kernel-trace summary of the bench.
# usage (on the GPU box): bash tools/gpu_round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu --steps 3 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
echo prof_ok
