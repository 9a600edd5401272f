#!/bin/bash
# Parity tests on the default build, then A/B of alternative builds (FMX_LIB) pipelined and isolated.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
if [ -x tools/ubench/constrain ]; then timeout -k 10 120 tools/ubench/constrain || exit 1; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
L=$PWD/fmtuner-sdr_amd
bash tools/gpu_ab.sh ${AB_SPECS:-base:FMX_LIB=$L/libfmx_base.so new nofract:FMX_LIB=$L/libfmx_nofract.so base2:FMX_LIB=$L/libfmx_base.so new2 \
  sbase:FMX_LIB=$L/libfmx_base.so,FMX_SERIAL=1 snew:FMX_SERIAL=1 snofract:FMX_LIB=$L/libfmx_nofract.so,FMX_SERIAL=1}
