#!/usr/bin/env python3
"""Per-kernel sums of arbitrary PMC passes over the last frame of a bench run
(the dispatches after the last-but-one reduce_kernel, counting kernels
excluded), plus derived unit utilisations:
  ta_busy   = TA_TA_BUSY_sum / n_cu / (GRBM_GUI_ACTIVE / 8)   (TA per CU)
  td_busy   = TD_TD_BUSY_sum / n_cu / (GRBM_GUI_ACTIVE / 8)
  l1_hit    = 1 - TCP_TCC_READ_REQ_sum / TCP_TOTAL_CACHE_ACCESSES_sum
  l2_hit    = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md "DVFS".)
usage: python3 tools/pmc_passes.py DIR_WITH_pN_SUBDIRS > out.json"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic_summary import last_frame, load  # noqa: E402

N_CU = 256


def main():
    pdir = sys.argv[1]
    per = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> sum over the frame (same pass)
    for p in sorted(os.listdir(pdir)):
        full = os.path.join(pdir, p)
        if not os.path.isdir(full):
            continue
        rows = load(full)
        if not rows:
            continue
        frame, _ = last_frame(rows)
        # GRBM_GUI_ACTIVE per pass: each pass carries its own (kernels re-run)
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d not in frame:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[name][r["Counter_Name"] + "@" + p] += float(r["Counter_Value"])
    out = {}
    for k, c in per.items():
        e = {}
        for key, v in c.items():
            e[key] = v
        # derived, within one pass (same dispatches)
        for p in {key.split("@")[1] for key in c}:
            g = c.get("GRBM_GUI_ACTIVE@" + p)
            if not g:
                continue
            cyc = g / 8.0
            e["cycles@" + p] = cyc
            for ctr, nm in (("TA_TA_BUSY_sum", "ta_busy"), ("TD_TD_BUSY_sum", "td_busy"),
                            ("TCP_TCP_TA_DATA_STALL_CYCLES_sum", "tcp_ta_data_stall"),
                            ("TCP_PENDING_STALL_CYCLES_sum", "tcp_pending_stall"),
                            ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "ta_addr_stalled_by_tc"),
                            ("TD_TC_STALL_sum", "td_tc_stall")):
                v = c.get(ctr + "@" + p)
                if v is not None:
                    e[nm] = round(v / N_CU / cyc, 4)
        acc = next((v for key, v in c.items() if key.startswith("TCP_TOTAL_CACHE_ACCESSES_sum@")), None)
        req = next((v for key, v in c.items() if key.startswith("TCP_TCC_READ_REQ_sum@")), None)
        if acc and req is not None:
            e["l1_hit_est"] = round(1.0 - req / acc, 4)
        h = next((v for key, v in c.items() if key.startswith("TCC_HIT_sum@")), None)
        m = next((v for key, v in c.items() if key.startswith("TCC_MISS_sum@")), None)
        if h is not None and m:
            e["l2_hit"] = round(h / (h + m), 4)
        out[k] = e
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
