#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_traffic.sh for the LAST frame of
the bench run (the kernels after the last-but-one reduce_kernel).

HBM bytes = FETCH_SIZE x 2 (gfx950 reports half the bytes of wide reads,
MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KB per dispatch.  Our loads
are mostly 8-byte (FP64) per lane, an access width the guide calls
uncalibrated, so the figure is an estimate; ratios between runs are sound.
Writes profiles/traffic_<tag>.json and profiles/traffic_latest.json (read by
bench.py for roofline.traffic)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(pdir):
    f = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return []
    rows = list(csv.DictReader(open(f[0])))
    return rows


def last_frame(rows):
    """dispatch ids of the last frame: after the last-but-one reduce_kernel"""
    disp = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        disp[d] = r["Kernel_Name"]
    ids = sorted(disp)
    red = [d for d in ids if disp[d].startswith("reduce_kernel")]
    lo = red[-2] if len(red) >= 2 else -1
    hi = red[-1] if red else ids[-1]
    return {d for d in ids if lo < d <= hi and "<true" not in disp[d]}, disp


def main():
    pdir, tag = sys.argv[1], sys.argv[2]
    per_ctr = defaultdict(lambda: defaultdict(float))  # ctr -> kernel -> sum
    tot = defaultdict(float)
    for p in sorted(glob.glob(os.path.join(pdir, "p*"))):
        if not os.path.isdir(p):
            continue
        rows = load(p)
        if not rows:
            continue
        frame, disp = last_frame(rows)
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d not in frame:
                continue
            name = r["Kernel_Name"].split("(")[0]
            v = float(r["Counter_Value"])
            per_ctr[r["Counter_Name"]][name] += v
            tot[r["Counter_Name"]] += v
    fetch = tot.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = tot.get("WRITE_SIZE", 0.0) * 1024
    import hashlib
    lib = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "lib", "librtx_hip.so")
    bid = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "lib", "BUILD_ID")
    out = {
        "tag": tag, "flags": "-w 1920 -r 5 -O r -A 4", "n_gpus": 1,
        # the build the counters were taken on (bench.py uses the file only
        # for the same librtx_hip.so)
        "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
        "build_id": open(bid).read().strip() if os.path.exists(bid) else None,
        "unit_of_launch": "frame (all kernels of one frame; bench.py roofline is per frame)",
        "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "fetch_correction": "FETCH_SIZE x 2 (gfx950, MI355X_MICROARCH.md HBM section); 8-B/lane loads uncalibrated",
        "l2_hit_rate": (tot["TCC_HIT_sum"] / (tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"])
                        if tot.get("TCC_HIT_sum", 0) + tot.get("TCC_MISS_sum", 0) > 0 else None),
        "per_kernel": {c: dict(k) for c, k in per_ctr.items()},
        "totals": dict(tot),
    }
    sq = tot.get("SQ_WAVE_CYCLES", 0.0)
    if sq:
        out["sq_fractions"] = {k: tot.get(k, 0.0) / sq for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                  "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for path in (os.path.join("profiles", f"traffic_{tag}.json"), os.path.join("profiles", "traffic_latest.json"),
                 os.path.join("gpurun_out", f"traffic_{tag}.json")):  # (gpurun_out/ comes back from the box)
        with open(os.path.join(ROOT, path), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_read_bytes_per_launch", "hbm_write_bytes_per_launch",
                                          "l2_hit_rate")}), out.get("sq_fractions"))


if __name__ == "__main__":
    main()
