#!/bin/bash
# Kernel timeline of the pipelined bench (rocprofv3 kernel trace) -> per-step
# overlap summary (tools/timeline.py).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/timeline
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/err.txt" || exit 1
python3 "$ROOT/tools/timeline.py" "$OUT" | tee "$OUT/summary.txt"
