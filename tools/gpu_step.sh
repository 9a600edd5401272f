#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu_iso.sh 20 base cur
bash tools/gpu_abn.sh 3 100 base cur > gpurun_out/abn.log 2>&1; tail -2 gpurun_out/abn.log
