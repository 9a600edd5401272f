#!/bin/bash
# GPU parity tests + bench (pipelined and step-synchronized) on the box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --sync-steps > gpurun_out/bench_sync.json 2>> gpurun_out/bench.err
