#!/bin/bash
# round-6 GPU session 24: k_pll's blend-smoother wave at index 4 (it shares
# W0's SIMD; every P wave then shares a SIMD with another P wave) -- parity
# suites on that library, step-time A/B at 4096 / 2048 channels, the last
# step's tail in a kernel trace
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_wb4.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipelined.py \
  tests/test_gpu_determinism.py tests/test_gpu_cfg4_sizes.py -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "not graft_smoke" > $O/tests_r06v.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_r06v.log | tail -6; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/gpu_abn.sh 5 20 cur wb4 > $O/ab4096_r06v.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06v.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur wb4 > $O/ab2048_r06v.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06v.txt
