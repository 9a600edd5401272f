"""Front-end kernel gaps and the ops between them, from a rocprofv3
--kernel-trace --memory-copy-trace CSV directory (tools/gpu_trace.sh)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
ks = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
ms = list(csv.DictReader(open(mc[0]))) if mc else []
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:28]) for k in ks]
ev += [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "copy " + m["Direction"][12:]) for m in ms]
ev.sort()
fe = [e for e in ev if "k_fe8" in e[2]]
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(fe, fe[1:])]
print("front-end launches", len(fe), "avg us", sum((e[1] - e[0]) for e in fe) / max(1, len(fe)) / 1e3)
print("gaps between front ends (us):", " ".join("%.1f" % g for g in gaps[-12:]))
if len(fe) > 4:
    a, b = fe[-4], fe[-3]
    for e in ev:
        if a[0] <= e[0] < b[0] + 1:
            print("  %9.1f %8.1f %s" % ((e[0] - a[0]) / 1e3, (e[1] - e[0]) / 1e3, e[2]))

# per kernel: mean duration and mean idle gap between consecutive launches
import statistics
print("kernel            n    dur_us   median gap_us (start[k+1] - end[k])")
for key in ("k_fe8", "k_pilot", "k_pll", "k_rs", "k_rds", "k_audio"):
    ks_ = [e for e in ev if key in e[2]]
    if len(ks_) < 3:
        continue
    ks_ = ks_[2:]  # skip warmup
    d = sum(e[1] - e[0] for e in ks_) / len(ks_) / 1e3
    gp = [(b[0] - a[1]) / 1e3 for a, b in zip(ks_, ks_[1:])]
    print("%-12s %5d %9.1f %8.1f" % (key, len(ks_), d, statistics.median(gp)))
if len(fe) > 3:
    print("step (front-end start to start, median) us: %.1f" % statistics.median(
        (b[0] - a[0]) / 1e3 for a, b in zip(fe[2:], fe[3:])))
# the front-end stream with k_pilot behind k_fe8 (round 4): k_fe8 end ->
# k_pilot start, k_pilot end -> next k_fe8 start
pil = [e for e in ev if "k_pilot" in e[2]]
if len(pil) > 3 and len(fe) > 3:
    g1, g2 = [], []
    for a, b in zip(fe[2:], fe[3:]):
        p = next((e for e in pil if a[1] <= e[0] < b[0]), None)
        if p:
            g1.append((p[0] - a[1]) / 1e3)
            g2.append((b[0] - p[1]) / 1e3)
    if g1:
        print("front-end stream gaps (median us): k_fe8 -> k_pilot %.1f, k_pilot -> k_fe8 %.1f" % (
            statistics.median(g1), statistics.median(g2)))

# per step (k-th launch of each kernel = step k): start / end of every kernel
# relative to its front end's start, us -- which stream waits for which
KEYS = ("k_fe8", "k_pilot", "k_pll", "k_rs", "k_rds", "k_audio")
seq = {key: [e for e in ev if key in e[2]] for key in KEYS}
# the first block runs k_frontend (cold decimator history), later ones k_fe8:
# the i-th front end of any kind is step i
seq["k_fe8"] = [e for e in ev if "k_fe8" in e[2] or "k_frontend" in e[2]]
# a k_frontend step (the first, cold history) runs its own pilot BPF and RDS
# resampler: k_pilot / k_rs of step k = the next launch starting after that
# step's k_fe8 ended
for key in ("k_pilot", "k_rs"):
    lst, out, j = seq[key], [], 0
    for f in seq["k_fe8"]:
        if "k_frontend" in f[2]:
            out.append(None)
            continue
        while j < len(lst) and lst[j][0] < f[1]:
            j += 1
        out.append(lst[j] if j < len(lst) else None)
        j += 1
    seq[key] = out
KEYS = tuple(k for k in KEYS if seq[k])
nst = min(len(seq[k]) for k in KEYS)
while nst > 0 and any(seq[k][nst - 1] is None for k in KEYS):
    nst -= 1  # the trace's last steps may end before their k_pilot / k_rs
if nst > 6:
    print("step  " + "".join("%-16s" % (k[2:] + "[s,e]") for k in KEYS) + "(us from fe start)")
    for k in range(nst - 8, nst):
        t0 = seq["k_fe8"][k][0]
        row = " ".join("%6.0f,%6.0f " % ((seq[key][k][0] - t0) / 1e3, (seq[key][k][1] - t0) / 1e3)
                       if seq[key][k] else "     -,     - " for key in KEYS)
        print("%4d  %s" % (k, row))
