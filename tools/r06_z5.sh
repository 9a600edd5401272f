#!/bin/bash
# round-6 GPU session 31: k_rs part size below 4096 channels -- 3 / 6 tiles
# per workgroup under 2048 channels (rss3, rss6), 6 / 12 at 2048 (m6, m12)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_AB_ARGS="--channels 1024" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur rss6 rss3 > $O/ab1024_r06z5.txt 2>&1 || exit 3
tail -3 $O/ab1024_r06z5.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur m6 m12 > $O/ab2048_r06z5.txt 2>&1 || exit 3
tail -3 $O/ab2048_r06z5.txt
