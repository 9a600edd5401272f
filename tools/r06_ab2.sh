#!/bin/bash
# round-6 GPU session: full GPU tests of the tree (k_fe8 with the LDS tap
# window), the PLL-form parity A/B, then step-time A/Bs at 2048 / 4096
# channels of r05 (HEAD of round 5), cur and the PLL forms
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/tests_r06b.log 2>&1
rc=$?; tail -4 $O/tests_r06b.log; [ $rc -le 1 ] || exit $rc
bash tools/pll_forms_ab.sh cur c1 c2 c3 c3w c1w > $O/pllab_summary.txt 2>&1; rc=$?
cat $O/pllab_summary.txt; [ $rc -le 1 ] || exit $rc
FMX_AB_ARGS="--channels 2048" timeout -k 10 600 bash tools/gpu_abn.sh 3 20 r05 cur nopq c1 c3 c3w > $O/ab2048_r06b.txt 2>&1 || exit 3
tail -7 $O/ab2048_r06b.txt
timeout -k 10 600 bash tools/gpu_abn.sh 3 20 r05 cur nopq c1 c3 c3w > $O/ab4096_r06b.txt 2>&1 || exit 3
tail -7 $O/ab4096_r06b.txt
