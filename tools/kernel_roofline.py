#!/usr/bin/env python3
"""Per-kernel roofline of the headline frame: each kernel class's algorithmic
bytes (bench.py's work.kernels, from rtx_last_work) over that class's launch
time in a rocprofv3 --stats summary of the same build (non-counting
instantiations only), and its PMC-measured HBM bytes (traffic file, FETCH x 2
+ WRITE) over the same time.

  closest — trace_kernel<false, 1, ...>  (camera / reflection / refraction
            queries and, on fused frames, their shading)
  next    — trace_kernel<false, 2, ...>  (shadow walks)
  tail    — tail_fused_kernel<false> / tail_kernel<false, ...>
The classes run concurrently on 3 streams, so each class's time is the sum of
its launch durations: achieved = bytes per launch / average launch duration.

usage: kernel_roofline.py BENCH.json KERNEL_STATS.csv FRAMES [TRAFFIC.json]"""
import csv
import json
import sys

HBM_PEAK_GBS = 8000.0
CLASSES = {"closest": ("trace_kernel<false, 1,",), "next": ("trace_kernel<false, 2,",),
           "tail": ("tail_fused_kernel<false>", "tail_kernel<false,")}


def main():
    bench = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    rows = list(csv.DictReader(open(sys.argv[2])))
    frames = float(sys.argv[3])
    traffic = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else None
    work = bench["work"]["kernels"]
    out = {"build": bench.get("build"), "frames_profiled": frames, "classes": {}}
    for c, pats in CLASSES.items():
        ms = sum(float(r["TotalDurationNs"]) for r in rows if any(r["Name"].startswith("void " + p) for p in pats))
        calls = sum(int(r["Calls"]) for r in rows if any(r["Name"].startswith("void " + p) for p in pats))
        ms = ms / 1e6 / frames
        w = work.get(c, {})
        b = w.get("algorithmic_bytes", 0)
        e = {"ms_per_frame": round(ms, 3), "launches_per_frame": calls / frames,
             "avg_launch_us": round(ms * 1e3 / (calls / frames), 1) if calls else None,
             "algorithmic_bytes": b, "achieved_gbs": round(b / (ms * 1e-3) / 1e9, 1) if ms else None,
             "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ms else None, "work": w}
        if traffic and ms:
            pk = traffic.get("per_kernel", {})
            hb = 0.0
            for ctr, scale in (("FETCH_SIZE", 2048.0), ("WRITE_SIZE", 1024.0)):
                hb += scale * sum(v for k, v in pk.get(ctr, {}).items()
                                  if any(k.startswith("void " + p) for p in pats))
            e["hbm_bytes_measured"] = hb
            e["frac_hbm_measured"] = round(hb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            def cls_sum(ctr):
                return sum(v for k, v in pk.get(ctr, {}).items() if any(k.startswith("void " + p) for p in pats))
            valu = cls_sum("SQ_INSTS_VALU")
            if valu:
                # SIMD cycles: 2 per wave64 VALU instruction on a 32-lane CDNA4
                # SIMD, 4 for FP64 (half rate) — MI355X_MICROARCH.md
                f64 = sum(cls_sum(c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                               "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
                e["valu_insts"] = valu
                e["valu_f64_insts"] = f64
                e["frac_valu"] = round((2 * (valu - f64) + 4 * f64) / (ms * 1e-3) / (256 * 4 * 2.4e9), 4)
        out["classes"][c] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
