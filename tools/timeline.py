#!/usr/bin/env python3
"""Kernel timeline of one rendered frame from a rocprofv3 kernel trace
(--kernel-trace --output-format csv): frames are cut at reduce_kernel; for
the frame chosen (default: the last) prints every launch's start offset,
duration, queue and grid, then per-kernel totals and the span of the tail.
usage: python tools/timeline.py <run_kernel_trace.csv> [frame_index] [--brief]"""
import csv
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n[:48]


def main():
    path = sys.argv[1]
    args = [a for a in sys.argv[2:] if not a.startswith("--")]
    brief = "--brief" in sys.argv
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    if not rows:
        print("no rows")
        return
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], []
    for r in rows:
        cur.append(r)
        if r["Kernel_Name"].startswith("reduce_kernel"):
            frames.append(cur)
            cur = []
    if cur:
        frames.append(cur)
    fi = int(args[0]) if args else -1
    fr = [r for r in frames[fi] if not r["Kernel_Name"].startswith("__amd") and "at::native" not in r["Kernel_Name"]]
    t0 = int(fr[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in fr)
    print(f"frames {len(frames)}; frame {fi}: {len(fr)} launches, span {(t1 - t0) / 1e6:.3f} ms")
    tot = {}
    for r in fr:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        tot.setdefault(k, [0, 0.0, 0.0])
        tot[k][0] += 1
        tot[k][1] += d
        tot[k][2] = max(tot[k][2], d)
        if not brief:
            q = r.get("Queue_Id", r.get("Stream_Id", "?"))
            g = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
            print(f"  {s:9.1f} us  {d:9.1f} us  q{q:>3}  grid {g:>9}  {k}")
    print("per kernel: calls, total us, max us")
    for k, (c, t, m) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"  {c:4d} {t:10.1f} {m:9.1f}  {k}")


if __name__ == "__main__":
    main()
