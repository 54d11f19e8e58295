set -o pipefail
cd $GRAFT_REPO_ROOT
V=cs378hgraphics-raytracer_amd/lib/variants
for cfg in "RTX_GROUPS=3 RTX_SLOTS=12582912" "RTX_GROUPS=4 RTX_SLOTS=16777216" "RTX_GROUPS=4 RTX_SLOTS=8388608" "RTX_GROUPS=3 RTX_SLOTS=12582912 RTX_HIP_LIB=$V/librtx_hip_t3a1.so" "RTX_GROUPS=3 RTX_SLOTS=12582912 RTX_HIP_LIB=$V/librtx_hip_t5a1.so"; do
  env RTX_WAVEFRONT=1 $cfg timeout -k 10 200 python bench.py --no-cpu --steps 2 > gpurun_out/exp.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/exp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_kernel_ms"])')"
done
