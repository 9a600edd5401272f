#!/usr/bin/env python3
"""Per-launch HBM-side bytes of each fmx kernel from the L2's memory-side
request counters BY REQUEST SIZE (round 6), instead of FETCH_SIZE's fixed
64 B per request:

  read bytes  = 32 TCC_EA0_RDREQ_32B + 64 TCC_EA0_RDREQ_64B + 128 TCC_EA0_RDREQ_128B
  write bytes = 64 TCC_EA0_WRREQ_64B + 32 (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)

FETCH_SIZE counts every read request as 64 B; the guide's x2 for it holds for
wide coalesced streams (all 128-B requests) only, so a kernel whose loads
split into 64-B or 32-B requests (k_rs's 64-B window segments, k_rds's dword
moves) was over-counted by the doubling (MI355X_MICROARCH.md "HBM [CDNA4]":
other access widths are uncalibrated).  Also reports each kernel's request
mix.

usage: pmc_reqsize.py OUT_JSON DIR [DIR ...]   (rocprofv3 --pmc output dirs)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

NAMES = ("k_fe8", "k_frontend", "k_pll", "k_pilot", "k_audio", "k_rds", "k_rs", "k_bits")


def short(name):
    for k in NAMES:
        if k + "<" in name or k + "(" in name or name.endswith(k):
            return k
    return None


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    val = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row["Kernel_Name"])
                    if k:
                        val[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"source": "rocprofv3 --pmc TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum / TCC_EA0_WRREQ{,_64B}_sum passes, "
                     "per launch (mean over dispatches)", "kernels": {}}
    for k, cs in sorted(val.items()):
        m = {c.replace("TCC_EA0_", "").replace("_sum", ""): sum(v) / len(v) for c, v in cs.items() if v}
        ent = dict(m)
        if all(x in m for x in ("RDREQ_32B", "RDREQ_64B", "RDREQ_128B")):
            ent["read_bytes"] = 32 * m["RDREQ_32B"] + 64 * m["RDREQ_64B"] + 128 * m["RDREQ_128B"]
            ent["fetch_size_equiv_x2"] = 2 * 64 * m.get("RDREQ", 0.0)  # what FETCH_SIZE x 2 would say
        if "WRREQ" in m and "WRREQ_64B" in m:
            ent["write_bytes"] = 64 * m["WRREQ_64B"] + 32 * (m["WRREQ"] - m["WRREQ_64B"])
        if "read_bytes" in ent and "write_bytes" in ent:
            ent["hbm_bytes"] = ent["read_bytes"] + ent["write_bytes"]
        res["kernels"][k] = ent
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, e in res["kernels"].items():
        print(k, {x: (round(y / 1e6, 2) if "bytes" in x or "x2" in x else round(y)) for x, y in e.items()})


if __name__ == "__main__":
    main()
