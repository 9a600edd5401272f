#!/bin/bash
# Round-end evidence on the GPU box: parity tests, smoke, rocprofv3 kernel
# stats + HBM PMC passes (tools/gpu_profile.sh), then the default bench line
# (with the CPU baseline) using the fresh PMC traffic.  Usage: tools/gpu_round.sh TAG
set -e
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
bash tools/gpu_profile.sh "$TAG" 10 > gpurun_out/profile_$TAG.log 2>&1
timeout -k 10 300 python bench.py --pmc-json gpurun_out/prof_$TAG/pmc_frontend.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
