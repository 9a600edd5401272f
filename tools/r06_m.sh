#!/bin/bash
# round-6 GPU session 13: the pilot BPF back inside k_fe8 (its RS = true
# instance with the resampler left to k_rs; no k_pilot) -- parity suites and
# step-time A/B (fp), k_rs at 4 parts (rs46) at 4096 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_fp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_pipelined.py tests/test_gpu_cfg4_sizes.py tests/test_gpu_determinism.py -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/tests_fp.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_fp.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur fp rs46 > $O/ab4096_fp.txt 2>&1 || exit 3
tail -3 $O/ab4096_fp.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur fp > $O/ab2048_fp.txt 2>&1 || exit 3
tail -2 $O/ab2048_fp.txt
