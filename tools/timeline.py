#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py: per-step start/end of each
fmx kernel relative to the step's frontend start (microseconds)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        name = r["Kernel_Name"]
        for k in ("k_frontend", "k_pll", "k_audio", "k_rds"):
            if k in name:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
fe = [r for r in rows if r[2] == "k_frontend"]
print("step  " + "  ".join(f"{k:>18s}" for k in ("k_frontend", "k_pll", "k_audio", "k_rds")))
for i, (s0, e0, _) in enumerate(fe[:-1]):
    s1 = fe[i + 1][0]
    seg = [r for r in rows if s0 <= r[0] < s1]
    out = []
    for k in ("k_frontend", "k_pll", "k_audio", "k_rds"):
        ks = [r for r in seg if r[2] == k]
        out.append(f"{(ks[0][0]-s0)/1e3:7.0f}..{(ks[0][1]-s0)/1e3:7.0f}" if ks else " " * 16)
    print(f"{i:4d}  " + "  ".join(f"{o:>18s}" for o in out) + f"   next fe +{(s1-s0)/1e3:.0f}")
