#!/bin/bash
# round-6 GPU session 7: the pilot BPF split between the front-end and the
# PLL stream (sp25 / sp40 / sp50: that percentage of the channels on sB), and
# k_pilot at wave priority 2 (pp2)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur sp25 sp40 sp50 pp2 > $O/ab4096_r06g.txt 2>&1 || exit 3
tail -5 $O/ab4096_r06g.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur sp25 sp50 > $O/ab2048_r06g.txt 2>&1 || exit 3
tail -3 $O/ab2048_r06g.txt
