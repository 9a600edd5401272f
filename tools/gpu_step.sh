#!/bin/bash
# scratch GPU step (edited per experiment)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 200 python tools/gpu_determinism.py 4096 8 1 > gpurun_out/det_cur.log 2>&1; echo "cur rc=$? $(tail -2 gpurun_out/det_cur.log)"
FMX_DIAG_NO_FE8=1 RDS_STAGE=0 timeout -k 10 200 python tools/gpu_determinism.py 4096 8 1 > gpurun_out/det_nofe8.log 2>&1; echo "nofe8 $(tail -1 gpurun_out/det_nofe8.log)"
STEREO=0 RDS_STAGE=0 timeout -k 10 200 python tools/gpu_determinism.py 4096 8 1 > gpurun_out/det_mono.log 2>&1; echo "mono $(tail -1 gpurun_out/det_mono.log)"
exit 0
