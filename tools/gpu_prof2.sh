#!/bin/bash
# Round-2 profile set: kernel trace + stats, FETCH/WRITE PMC passes (per-kernel
# HBM bytes), two SQ counter passes.  Usage: tools/gpu_prof2.sh TAG
TAG=${1:-r02a}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
bash tools/gpu_profile.sh "$TAG" 10 > gpurun_out/profile_$TAG.log 2>&1 || { tail -20 gpurun_out/profile_$TAG.log; exit 1; }
tail -3 gpurun_out/profile_$TAG.log
bash tools/gpu_counters.sh "$TAG" > gpurun_out/counters_$TAG.log 2>&1 || { tail -20 gpurun_out/counters_$TAG.log; exit 1; }
cat gpurun_out/cnt_$TAG/summary.txt
