#!/bin/bash
# Where a latency-bound launch's wave time goes (GPU box): one PMC pass of
# SQ wave-state and instruction-fetch counters over an 8-way headline shard
# (tools/shard_probe.py --rank R), with the kernel trace, then per dispatch of
# the last frame: duration, effective clock (GRBM_GUI_ACTIVE / 8 / duration),
# waves, and the shares of wave time parked on waitcnt (SQ_WAIT_ANY), stalled
# at issue (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), with the
# instruction-cache misses per wave.
# usage: bash tools/pmc_tail.sh TAG [RANK] [N] [extra env VAR=value ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
RANK=${2:-6}
N=${3:-8}
shift 3 2>/dev/null
mkdir -p gpurun_out
OUT=gpurun_out/tail_${TAG}
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQC_ICACHE_MISSES GRBM_GUI_ACTIVE"
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
  env "$@" timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $OUT -o run -- \
    python3 tools/shard_probe.py --rank $RANK $N > $OUT.log 2>&1) || { echo "FAIL"; tail -5 $OUT.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
cc = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
disp = {}
for r in csv.DictReader(open(kt)):
    disp[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
cnt = defaultdict(dict)
for r in csv.DictReader(open(cc)):
    cnt[int(r["Dispatch_Id"])][r["Counter_Name"]] = cnt[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
ids = sorted(i for i in cnt if i in disp)
# the last frame: from the last lane_init_kernel on
last = max(i for i in ids if "lane_init" in disp[i][0])
print("dispatch kernel dur_us clock_ghz waves wave_us wait_any wait_inst active icache_miss_per_wave ifetch_per_wave")
for i in ids:
    if i < last:
        continue
    name, t0, t1 = disp[i]
    c = cnt[i]
    short = name.split("(")[0].replace("void ", "")[:44]
    dur = (t1 - t0) / 1e3
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / max(1e-9, (t1 - t0)) if t1 > t0 else 0
    w = max(1.0, c.get("SQ_WAVES", 0))
    wc = c.get("SQ_WAVE_CYCLES", 0)
    f = lambda k: round(c.get(k, 0) / wc, 3) if wc else 0
    print(i, short, round(dur, 1), round(clk, 2), int(w), round(wc * 4 / w / max(clk, 1e-9) / 1e3, 1),
          f("SQ_WAIT_ANY"), f("SQ_WAIT_INST_ANY"), f("SQ_ACTIVE_INST_ANY"),
          round(c.get("SQC_ICACHE_MISSES", 0) / w, 1), round(c.get("SQ_IFETCH", 0) / w, 1))
PY
