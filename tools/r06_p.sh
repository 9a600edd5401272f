#!/bin/bash
# round-6 GPU session 16: k_rds tap columns in registers -- all eleven at two
# waves per SIMD (hreg2), the first 8 / 6 within the three-wave budget (h8,
# h6) -- step-time A/B at 2048 / 4096 / 1024 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 5 20 cur h8 h6 hreg2 > $O/ab2048_r06p.txt 2>&1 || exit 3
tail -4 $O/ab2048_r06p.txt
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur h8 h6 hreg2 > $O/ab4096_r06p.txt 2>&1 || exit 3
tail -4 $O/ab4096_r06p.txt
FMX_AB_ARGS="--channels 1024" timeout -k 10 700 bash tools/gpu_abn.sh 3 20 cur h8 hreg2 > $O/ab1024_r06p.txt 2>&1 || exit 3
tail -3 $O/ab1024_r06p.txt
