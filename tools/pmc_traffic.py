#!/usr/bin/env python3
"""Per-launch HBM traffic of each fmx kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]":
FETCH_SIZE / WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts
half the bytes of a wide coalesced streaming read, so it is doubled.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON --channels C --block B
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, counter):
    per = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                per[name].append(float(row["Counter_Value"]))
    return per


def short(name):
    for k in ("k_fe8", "k_frontend", "k_pll", "k_pilot", "k_audio", "k_rds", "k_rs", "k_reset", "k_synth"):
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--channels", type=int, required=True)
    ap.add_argument("--block", type=int, required=True)
    a = ap.parse_args()
    fe = load(a.fetch_dir, "FETCH_SIZE")
    wr = load(a.write_dir, "WRITE_SIZE")
    res = {"channels": a.channels, "block": a.block,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB -> bytes, FETCH x2 (gfx950)",
           "kernels": {}}
    for name in set(fe) | set(wr):
        k = short(name)
        if k is None or k == "k_synth":
            continue
        f = fe.get(name, [])
        w = wr.get(name, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        ent = res["kernels"].setdefault(k, {})
        ent.update({"launches_fetch": len(f), "launches_write": len(w),
                    "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                    "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0)})
    # the steady-state frontend is k_fe8 (k_frontend runs the first, partial-history call)
    for k in ("k_fe8", "k_frontend"):
        if k in res["kernels"]:
            res["hbm_bytes_per_launch"] = res["kernels"][k]["hbm_bytes_per_launch"]
            res["frontend_kernel"] = k
            break
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
