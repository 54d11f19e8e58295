#!/bin/bash
# PMC passes on the memory pipeline (TA / TD / TCP / TCC) over one bench
# frame, each pass its own run (rocprofv3 does not split passes); then
# tools/pmc_passes.py -> gpurun_out/units_<TAG>.json
# usage: bash tools/profile_units.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/units_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${@:-"--no-cpu --steps 1 --warmup 0"}
i=0
for ctr in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_READ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 \
    || { echo "pass $i failed ($ctr)"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_passes.py $OUT > gpurun_out/units_$TAG.json
