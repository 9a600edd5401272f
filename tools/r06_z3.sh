#!/bin/bash
# round-6 GPU session 28: k_audio as a grid of 1024 / 2048 workgroups looping
# over the channels (fewer k_audio waves in flight beside the front end) --
# parity suites on ag1024, step-time A/B at 4096 / 2048 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_ag1024.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipelined.py \
  tests/test_gpu_cfg4_sizes.py tests/test_signal_level.py -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "not graft_smoke" > $O/tests_r06z3.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_r06z3.log | tail -6; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur ag1024 ag2048 > $O/ab4096_r06z3.txt 2>&1 || exit 3
tail -3 $O/ab4096_r06z3.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur ag1024 > $O/ab2048_r06z3.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06z3.txt
