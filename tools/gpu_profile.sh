#!/bin/bash
# Profile the 1-GPU bench on the GPU box (run through gpurun from the repo root):
#   kernel trace + stats (csv), then one --pmc pass per HBM counter.
# Usage: tools/gpu_profile.sh TAG [STEPS]
set -e
TAG=${1:-r01}
STEPS=${2:-10}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$ROOT/bench.py" --steps "$STEPS" --warmup 3 --no-cpu-baseline > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_write.json" 2> "$OUT/write.err"
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/fetch" "$OUT/write" "$OUT/pmc_frontend.json" --channels 4096 --block 4096
