#!/bin/bash
# 1-GPU channel sweep of the bench (no CPU baseline): one JSON line per
# channel count into gpurun_out/sweep_TAG.jsonl.  Usage: tools/gpu_sweep.sh TAG [C ...]
set -e
TAG=${1:-r03a}
shift || true
SIZES=${*:-"256 1024 2048 4096 8192 16384"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
OUT=gpurun_out/sweep_$TAG.jsonl
: > "$OUT"
for C in $SIZES; do
  timeout -k 10 240 python bench.py --channels "$C" --steps 20 --warmup 5 --no-cpu-baseline >> "$OUT" 2> gpurun_out/sweep_${TAG}_$C.err
  python - "$OUT" <<'EOF'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: v["avg_ms"] for n, v in r["kernels"].items()}
print(r["config"]["channels_rank0"], r["value"], r["ms_per_step"], k, flush=True)
EOF
done
