#!/bin/bash
# Kernel + memory-copy timeline of a short bench run (no counters), and the
# gaps between consecutive front-end kernels.  Usage: tools/gpu_trace.sh TAG
TAG=${1:-trace}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$ROOT/gpurun_out/$TAG" -o run \
  -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline ${FMX_AB_ARGS:-} > "$ROOT/gpurun_out/${TAG}_bench.json" 2> "$ROOT/gpurun_out/$TAG.err" || exit 1
python3 "$ROOT/tools/trace_gaps.py" "$ROOT/gpurun_out/$TAG"
