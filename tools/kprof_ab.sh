set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in prev cur; do
  if [ $v = prev ]; then export RTX_HIP_LIB=$GRAFT_REPO_ROOT/cs378hgraphics-raytracer_amd/lib/variants/librtx_hip_prev.so; else unset RTX_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_$v -o run -- python3 bench.py --no-cpu --steps 5 > gpurun_out/kp_$v.log 2>&1 || exit 1
done
for v in prev cur; do f=$(find gpurun_out/kp_$v -name '*kernel_stats.csv' | head -1); echo "== $v"; cut -d, -f1-4 $f | head -8; done
