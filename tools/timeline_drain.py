#!/usr/bin/env python3
"""Fill and drain of the bench's timed region, from a rocprofv3 kernel trace
(tools/gpu_trace.sh): the last `steps` front ends are the timed ones; prints
the region's span against steps x the median front-end period, the first
step's ramp (only the front-end stream has work), and the tail after the
last front end -- each kernel of the last step, when it started and ended
relative to the end of the last k_pilot.

usage: timeline_drain.py TRACE_DIR [steps]"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
NAMES = ("k_fe8", "k_pilot", "k_pll", "k_rs", "k_rds", "k_bits", "k_audio")


def short(n):
    for k in NAMES:
        if k + "<" in n or k + "(" in n:
            return k
    return None


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
ev = [e for e in ev if e[2]]
per = {k: [e for e in ev if e[2] == k] for k in NAMES}
fe = per["k_fe8"][-steps:]
t0 = fe[0][0]
region = [e for e in ev if e[0] >= t0]
t_end = max(e[1] for e in region)
period = statistics.median((b[0] - a[0]) for a, b in zip(fe, fe[1:]))
print(f"timed region (first timed k_fe8 start -> last kernel end): {(t_end - t0) / 1e3:.1f} us for {steps} steps")
print(f"median front-end period {period / 1e3:.1f} us; {steps} x period = {steps * period / 1e3:.1f} us; "
      f"excess {(t_end - t0 - steps * period) / 1e3:.1f} us")
last_pilot = per["k_pilot"][-1]
print(f"first step: k_fe8 {(fe[0][1] - fe[0][0]) / 1e3:.1f} us (later median "
      f"{statistics.median(e[1] - e[0] for e in fe[1:]) / 1e3:.1f})")
print(f"tail after the last k_pilot end: {(t_end - last_pilot[1]) / 1e3:.1f} us")
for k in NAMES[2:]:
    if per[k]:
        s, e, _ = per[k][-1]
        print(f"  last {k:8s} start {(s - last_pilot[1]) / 1e3:+8.1f}  end {(e - last_pilot[1]) / 1e3:+8.1f}  "
              f"dur {(e - s) / 1e3:7.1f} us")
