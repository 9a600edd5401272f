#!/bin/bash
# round-6 GPU session 14: k_fe8's carried state by LDS-DMA with the first
# chunk (no setup load waits) -- front-end parity suites, stage clocks,
# step-time A/B against HEAD's library (pre) at 4096 / 2048 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fe8_cold.py tests/test_gpu_pipelined.py \
  tests/test_gpu_cfg4_sizes.py tests/test_gpu_determinism.py tests/test_gpu_weak_carrier.py -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/tests_r06n.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_r06n.log | tail -8; [ $rc -le 1 ] || exit $rc
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_serial_r06n.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/stamps_serial_r06n.txt | head -12
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 pre cur > $O/ab4096_r06n.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06n.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 pre cur > $O/ab2048_r06n.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06n.txt
