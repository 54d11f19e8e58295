#!/bin/bash
# PMC passes over the bench (one frame after warmup), run on the GPU box:
#   pass 1 FETCH_SIZE, pass 2 WRITE_SIZE (separate: TCC slot budget),
#   pass 3 TCC hit/miss, pass 4 SQ wave-cycle breakdown, pass 5 the VALU
#   instruction mix (FP64 add/mul/fma/transcendental, int, convert).
# Then tools/traffic_summary.py writes profiles/traffic_<TAG>.json.
# usage: bash tools/profile_traffic.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok ($ctr)"
done
python3 tools/traffic_summary.py $OUT $TAG
