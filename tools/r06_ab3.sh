#!/bin/bash
# round-6 GPU session 3: PLL word forms (fused add3 form) parity + timing,
# k_rs with 12-tile workgroups, k_pilot on a fifth stream
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
bash tools/pll_forms_ab.sh cur c1 c1x c1a > $O/pllab3_summary.txt 2>&1; rc=$?
cat $O/pllab3_summary.txt; [ $rc -le 1 ] || exit $rc
FMX_AB_ARGS="--channels 2048" timeout -k 10 600 bash tools/gpu_abn.sh 3 20 cur c1x c1a rs12 ps > $O/ab2048_r06c.txt 2>&1 || exit 3
tail -6 $O/ab2048_r06c.txt
timeout -k 10 600 bash tools/gpu_abn.sh 3 20 cur c1x c1a rs12 ps > $O/ab4096_r06c.txt 2>&1 || exit 3
tail -6 $O/ab4096_r06c.txt
