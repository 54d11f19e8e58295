set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "RTX_GROUPS=2 RTX_SLOTS=2097152" "RTX_GROUPS=2 RTX_SLOTS=8388608" "RTX_GROUPS=2 RTX_SLOTS=16777216" "RTX_GROUPS=3 RTX_SLOTS=3145728" "RTX_GROUPS=3 RTX_SLOTS=6291456" "RTX_GROUPS=3 RTX_SLOTS=12582912"; do
  env RTX_WAVEFRONT=1 $cfg timeout -k 10 200 python bench.py --no-cpu --steps 2 > gpurun_out/exp.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/exp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_kernel_ms"])')"
done
