#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
bash tools/gpu_abn.sh 2 100 cur f1:FMX_FE_PRIO=1 f2:FMX_FE_PRIO=2 f3:FMX_FE_PRIO=3 s0:FMX_SERIAL_PRIO=0 > gpurun_out/abn.log 2>&1; tail -5 gpurun_out/abn.log
