#!/bin/bash
# Quick GPU iteration: parity tests, pipelined bench, serialized-stream bench
# (FMX_SERIAL=1: every kernel on one stream, so its HIP-event time is isolated).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
FMX_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_serial.json 2>> gpurun_out/bench.err || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/bench.json", "gpurun_out/bench_serial.json"):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
