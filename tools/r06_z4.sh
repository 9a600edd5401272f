#!/bin/bash
# round-6 GPU session 30: k_rs in finer parts below 2048 channels (12 / 6
# tiles per workgroup; libraries built from a patched worktree) -- RDS parity
# at 1024 channels on rss12, step-time A/B at 1024 / 256 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_rss12.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "cfg5 or staggered" > $O/tests_r06z4.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_r06z4.log | tail -4; [ $rc -le 1 ] || exit $rc
FMX_AB_ARGS="--channels 1024" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur rss12 rss6 > $O/ab1024_r06z4.txt 2>&1 || exit 3
tail -3 $O/ab1024_r06z4.txt
FMX_AB_ARGS="--channels 256" timeout -k 10 700 bash tools/gpu_abn.sh 3 20 cur rss12 rss6 > $O/ab256_r06z4.txt 2>&1 || exit 3
tail -3 $O/ab256_r06z4.txt
