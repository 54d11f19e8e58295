set -o pipefail
cd $GRAFT_REPO_ROOT
V=cs378hgraphics-raytracer_amd/lib/variants
for cfg in "RTX_HIP_LIB=" "RTX_HIP_LIB=$V/librtx_hip_o2.so" "RTX_HIP_LIB=$V/librtx_hip_o2a3.so" "RTX_HIP_LIB=$V/librtx_hip_o2a4.so"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu --steps 3 > gpurun_out/exp.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/exp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/exp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_kernel_ms"])')"
done
