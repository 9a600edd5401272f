#!/bin/bash
# scratch GPU step (edited per experiment)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
bash tools/gpu_step2.sh
bash tools/gpu_trace.sh trace_r02d > gpurun_out/trace_r02d.txt 2>&1; tail -24 gpurun_out/trace_r02d.txt
