#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py: per-step start..end of each
fmx kernel relative to the step's front-end start (microseconds)."""
import csv
import glob
import os
import sys

KEYS = ("fe", "k_pll", "k_audio", "k_rds")
d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        name = r["Kernel_Name"]
        key = "fe" if ("k_fe8" in name or "k_frontend" in name) else next((k for k in KEYS[1:] if k in name), None)
        if key:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), key))
rows.sort()
fe = [r for r in rows if r[2] == "fe"]
print("step  " + "  ".join(f"{k:>16s}" for k in KEYS) + "   (us from the step's front-end start)")
for i, (s0, e0, _) in enumerate(fe[:-1]):
    s1 = fe[i + 1][0]
    out = []
    for k in KEYS:
        # the kernel of this step: the first launch of k starting after this front end
        ks = [r for r in rows if r[2] == k and r[0] >= s0]
        out.append(f"{(ks[0][0]-s0)/1e3:7.0f}..{(ks[0][1]-s0)/1e3:6.0f}" if ks else " " * 15)
    print(f"{i:4d}  " + "  ".join(f"{o:>16s}" for o in out) + f"   next fe +{(s1-s0)/1e3:.0f}")
