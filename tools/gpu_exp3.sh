set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -x -q -m gpu --tb=short > gpurun_out/pytest_paths.log 2>&1; echo pytest_rc=$?; tail -5 gpurun_out/pytest_paths.log
for cfg in "RTX_WAVEFRONT=1 RTX_GROUPS=1 RTX_SLOTS=8388608" "RTX_WAVEFRONT=1 RTX_GROUPS=4 RTX_SLOTS=2097152" "RTX_WAVEFRONT=1 RTX_GROUPS=4 RTX_SLOTS=4194304" "RTX_WAVEFRONT=1 RTX_GROUPS=4 RTX_SLOTS=8388608" "RTX_WAVEFRONT=1 RTX_GROUPS=8 RTX_SLOTS=4194304" "RTX_WAVEFRONT=1 RTX_GROUPS=2 RTX_SLOTS=4194304"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu --steps 2 > gpurun_out/exp.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/exp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_kernel_ms"], d["roofline"]["launches_per_frame"])')"
done
