set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "RTX_WAVEFRONT=1 RTX_SLOTS=4194304" "RTX_WAVEFRONT=1 RTX_SLOTS=8388608" "RTX_WAVEFRONT=1 RTX_SLOTS=16777216" "RTX_WAVEFRONT=1 RTX_SLOTS=33554432"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu --steps 2 > gpurun_out/exp.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/exp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_kernel_ms"], d["roofline"]["launches_per_frame"])')"
done
