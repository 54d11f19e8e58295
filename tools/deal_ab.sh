# Parity suite, then an A/B of the tile deal on the shard probe (same box):
# default (rotated rows) vs the column-deal variant build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_ab.log 2>&1; rc=$?
echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu_ab.log
[ $rc -eq 0 ] || exit 1
O=gpurun_out/deal_ab.txt; : > $O
echo "== rotated" >> $O
timeout -k 10 200 python -u tools/shard_probe.py ${NS:-1 2 4 8} 2>/dev/null >> $O || exit 1
echo "== columns" >> $O
RTX_HIP_LIB=$PWD/cs378hgraphics-raytracer_amd/lib/variants/librtx_hip_cols.so timeout -k 10 200 python -u tools/shard_probe.py ${NS:-2 4 8} 2>/dev/null >> $O || exit 1
cat $O
