#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy of librtx_hip from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (a saved stderr file).
usage: python tools/kres.py REMARKS.txt [substring ...]"""
import re
import sys

def main():
    txt = open(sys.argv[1]).read().splitlines()
    filt = sys.argv[2:]
    cur = None
    rows = []
    for ln in txt:
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, ln)
            if m:
                cur[key] = int(m.group(1))
    for r in rows:
        if filt and not any(f in r["name"] for f in filt):
            continue
        print(f"{r.get('vgpr', '?'):>4} v {r.get('agpr', 0):>2} a {r.get('scratch', '?'):>4} B scr occ {r.get('occ', '?')}  {r['name'][:110]}")

if __name__ == "__main__":
    main()
