#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_MFMA / LDS instructions per k_fe8 launch for library variants (one rocprofv3
# --pmc pass each, synchronized bench, 2048 channels): tools/gpu_valu_ab.sh name...
# (name "cur" = libfmx.so, else fmtuner-sdr_amd/libfmx_<name>.so)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/valu_ab
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib=$ROOT/fmtuner-sdr_amd/libfmx.so; [ "$v" = cur ] || lib=$ROOT/fmtuner-sdr_amd/libfmx_$v.so
  FMX_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d "$OUT/$v" -o run \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --sync-steps --channels 2048 > "$OUT/$v.json" 2> "$OUT/$v.err" || exit 1
  python3 - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_fe8" in r["Kernel_Name"] or "k_pilot" in r["Kernel_Name"]:
            k = "k_fe8" if "k_fe8" in r["Kernel_Name"] else "k_pilot"
            per[(k, r["Counter_Name"], r.get("Dispatch_Id", ""))] += float(r["Counter_Value"])
    for (k, c, _), x in per.items():
        acc[k][c].append(x)
for k in sorted(acc):
    print(sys.argv[2], k, {c: round(sum(v) / len(v) / 1e6, 3) for c, v in sorted(acc[k].items())})
PY
done
