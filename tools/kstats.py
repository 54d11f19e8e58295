#!/usr/bin/env python3
"""Per-frame kernel time summary of a rocprofv3 --stats csv.
usage: kstats.py run_kernel_stats.csv FRAMES"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frames = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = 0.0
for r in rows:
    ms = float(r["TotalDurationNs"]) / 1e6 / frames
    tot += ms
    print(f"{r['Name'][:70]:70s} calls/frame {int(r['Calls']) / frames:7.1f}  ms/frame {ms:8.2f}  avg_us {float(r['AverageNs']) / 1e3:8.1f}")
print(f"total kernel ms/frame {tot:.2f}")
