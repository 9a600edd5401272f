#!/bin/bash
# Stage clocks of k_fe8 / k_rds / k_pll waves.  Needs libfmx.so built with
# `make -C fmtuner-sdr_amd STAMPS=1 -B` (rebuild without STAMPS afterwards).
# Runs the pipelined streams and then FMX_SERIAL=1 (kernels in isolation).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/fe_stamps.py > gpurun_out/stamps.txt 2>&1 || exit 1
FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > gpurun_out/stamps_serial.txt 2>&1 || exit 1
echo "== pipelined"; grep -v amdgpu.ids gpurun_out/stamps.txt
echo "== serial"; grep -v amdgpu.ids gpurun_out/stamps_serial.txt
