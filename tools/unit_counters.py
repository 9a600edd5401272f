#!/usr/bin/env python3
"""Per-launch unit counters of each fmx kernel from rocprofv3 --pmc passes
(tools/gpu_units.sh), for bench.py's per-unit roofline ("units"):

  valu_insts            SQ_INSTS_VALU (wave-instructions, MFMA included)
  mfma_insts            SQ_INSTS_MFMA
  mfma_flop_f16 / _f32  SQ_INSTS_VALU_MFMA_MOPS_F16 / _F32 x 512 (FLOP)
  mfma_busy_cycles      SQ_VALU_MFMA_BUSY_CYCLES
  lds_insts             SQ_INSTS_LDS
  lds_active_cycles     SQ_LDS_IDX_ACTIVE (LDS-array cycles, all CUs)
  lds_bank_conflict     SQ_LDS_BANK_CONFLICT (extra cycles)
  gui_active            GRBM_GUI_ACTIVE (GPU cycles of the dispatch, max over XCDs)
  fetch_bytes           FETCH_SIZE KiB x 1024 x 2 (gfx950 counts half of a wide read)
  write_bytes           WRITE_SIZE KiB x 1024

Corrections per /opt/skills/guides/MI355X_MICROARCH.md ("HBM [CDNA4]",
"rocprofv3 PMC slots").  The library the passes ran (its SHA-256 prefix, from
the bench JSON each pass printed) is recorded, so bench.py can tell whether a
units file belongs to the library it loaded.

usage: unit_counters.py OUT_DIR OUT_JSON --channels C --block B
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

COUNTERS = {
    "SQ_INSTS_VALU": ("valu_insts", 1.0),
    "SQ_INSTS_MFMA": ("mfma_insts", 1.0),
    "SQ_INSTS_VALU_MFMA_MOPS_F16": ("mfma_flop_f16", 512.0),
    "SQ_INSTS_VALU_MFMA_MOPS_F32": ("mfma_flop_f32", 512.0),
    "SQ_VALU_MFMA_BUSY_CYCLES": ("mfma_busy_cycles", 1.0),
    "SQ_INSTS_LDS": ("lds_insts", 1.0),
    "SQ_LDS_IDX_ACTIVE": ("lds_active_cycles", 1.0),
    "SQ_LDS_BANK_CONFLICT": ("lds_bank_conflict", 1.0),
    "GRBM_GUI_ACTIVE": ("gui_active", 1.0),
    "FETCH_SIZE": ("fetch_bytes", 2.0 * 1024.0),
    "WRITE_SIZE": ("write_bytes", 1024.0),
}


def short(name):
    for k in ("k_fe8", "k_frontend", "k_pll", "k_pilot", "k_audio", "k_rds", "k_bits", "k_rs", "k_reset", "k_synth", "k_copy16"):
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("out")
    ap.add_argument("--channels", type=int, required=True)
    ap.add_argument("--block", type=int, required=True)
    a = ap.parse_args()
    # per (kernel, counter): values of every dispatch (a dispatch's rows per
    # counter are summed over dimensions first)
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(a.out_dir, "**", "*counter_collection.csv"), recursive=True):
        per_dispatch = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                c = row.get("Counter_Name")
                if c not in COUNTERS:
                    continue
                k = short(row["Kernel_Name"])
                if k is None:
                    continue
                per_dispatch[(k, c, row.get("Dispatch_Id", row.get("Correlation_Id", "")))] += float(row["Counter_Value"])
        for (k, c, _), v in per_dispatch.items():
            vals[(k, c)].append(v)
    libs = set()
    for jf in glob.glob(os.path.join(a.out_dir, "bench_*.json")):
        try:
            with open(jf) as fh:
                libs.add(json.load(fh)["library"]["sha256_16"])
        except (OSError, ValueError, KeyError):
            pass
    res = {"channels": a.channels, "block": a.block,
           "library_sha256_16": sorted(libs)[0] if len(libs) == 1 else sorted(libs),
           "source": "rocprofv3 --kernel-trace --pmc passes (tools/gpu_units.sh); per launch, mean over the dispatches",
           "kernels": {}}
    for (k, c), v in sorted(vals.items()):
        if k in ("k_synth", "k_reset", "k_copy16"):
            continue
        name, scale = COUNTERS[c]
        ent = res["kernels"].setdefault(k, {})
        ent[name] = scale * sum(v) / len(v)
        ent.setdefault("dispatches", {})[name] = len(v)
    for ent in res["kernels"].values():
        if "fetch_bytes" in ent and "write_bytes" in ent:
            ent["hbm_bytes"] = ent["fetch_bytes"] + ent["write_bytes"]
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
