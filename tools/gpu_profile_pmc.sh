#!/bin/bash
# Per-kernel HBM bytes per launch: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), then
# tools/pmc_traffic.py.  Usage: tools/gpu_profile_pmc.sh TAG
set -e
TAG=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_write.json" 2> "$OUT/write.err"
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/fetch" "$OUT/write" "$OUT/pmc_frontend.json" --channels 4096 --block 4096
cat "$OUT/pmc_frontend.json"
