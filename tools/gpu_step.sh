#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
bash tools/gpu_abn.sh 3 100 cur nb4 > gpurun_out/abn.log 2>&1; tail -2 gpurun_out/abn.log
