#!/bin/bash
# round-6 GPU session 19: non-temporal loads of the once-read streams (FMX_NT:
# nt1 = k_fe8's u8 IQ; nt15 = also k_rds's input, k_pll's pilot tiles,
# k_audio's raw L/R) -- step-time A/B at 4096 / 2048 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur nt1 nt15 > $O/ab4096_r06r.txt 2>&1 || exit 3
tail -3 $O/ab4096_r06r.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur nt1 nt15 > $O/ab2048_r06r.txt 2>&1 || exit 3
tail -3 $O/ab2048_r06r.txt
