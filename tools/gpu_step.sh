#!/bin/bash
# scratch GPU step (edited per experiment)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
L=$PWD/fmtuner-sdr_amd
for v in cur pk; do
  lib=$L/libfmx_$v.so; [ $v = cur ] && lib=$L/libfmx.so
  STEREO=0 RDS_STAGE=0 FMX_DIAG_RDS_DUMP=1 FMX_LIB=$lib timeout -k 10 200 python tools/gpu_determinism.py 4096 8 1 > gpurun_out/det_$v.log 2>&1; echo "$v dump rc=$? $(tail -1 gpurun_out/det_$v.log)"
done
timeout -k 10 200 python tools/gpu_determinism.py 4096 8 2 > gpurun_out/det_full.log 2>&1; echo "full rc=$? $(tail -1 gpurun_out/det_full.log)"
exit 0
