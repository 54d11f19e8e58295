#!/bin/bash
# One PMC pass (L2 hit/miss per kernel) over one bench frame for each
# configuration given as VAR=value[,VAR=value] (run on the GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/l2_${TAG}_$i -o run -- python3 bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/l2_${TAG}_$i.log 2>&1 || { echo "FAIL [$cfg]"; tail -5 gpurun_out/l2_${TAG}_$i.log; exit 1; }
  python3 - gpurun_out/l2_${TAG}_$i "$cfg" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    if "<true" in k or not ("trace" in k or "advance" in k):
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], {k: round(v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 3) for k, v in acc.items()})
PY
done
