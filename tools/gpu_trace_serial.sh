#!/bin/bash
# Kernel trace of the serialized-stream bench (FMX_SERIAL=1) for builds given as FMX_LIB tags
# (libfmx_<tag>.so, "default" = libfmx.so): per-kernel duration spread under rocprofv3.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for t in ${TR_TAGS:-default}; do
  lib=$ROOT/fmtuner-sdr_amd/libfmx.so; [ "$t" != default ] && lib=$ROOT/fmtuner-sdr_amd/libfmx_$t.so
  FMX_LIB=$lib FMX_SERIAL=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/trs_$t" -o run \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/trs_$t.json" 2> "$ROOT/gpurun_out/trs_$t.err" || exit 1
  python3 - "$ROOT/gpurun_out/trs_$t" "$t" <<'PY'
import csv, glob, sys, statistics as S
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = {}
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-12:]
    d.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n, v in d.items():
    if len(v) > 5:
        v = sorted(v)
        print(sys.argv[2], n, "n", len(v), "min %.3f med %.3f max %.3f" % (v[0], S.median(v), v[-1]))
PY
done
