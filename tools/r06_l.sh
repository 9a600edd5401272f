#!/bin/bash
# round-6 GPU session 12: the RDS resampler fused into k_rds (fz) -- the GPU
# parity suites through it (groups bit-exact), then step-time A/B against the
# current library at 4096 and 2048 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_fz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_pipelined.py tests/test_gpu_cfg4_sizes.py tests/test_gpu_determinism.py tests/test_gpu_weak_carrier.py \
  tests/test_gpu_fe8_cold.py -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_fz.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_fz.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur fz > $O/ab4096_fz.txt 2>&1 || exit 3
tail -2 $O/ab4096_fz.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur fz > $O/ab2048_fz.txt 2>&1 || exit 3
tail -2 $O/ab2048_fz.txt
