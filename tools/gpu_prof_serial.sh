#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_serial
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
FMX_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/err.txt"
cat "$OUT"/run_kernel_stats.csv | cut -c1-200
