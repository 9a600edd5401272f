#!/bin/bash
# round-6 GPU session 26: k_pll's serial waves (W0, WB) at priority 3 (above
# k_rds's 2) -- step-time A/B at 4096 / 2048 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 700 bash tools/gpu_abn.sh 5 20 cur sp3 > $O/ab4096_r06x.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06x.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 5 20 cur sp3 > $O/ab2048_r06x.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06x.txt
