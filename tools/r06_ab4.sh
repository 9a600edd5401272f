#!/bin/bash
# round-6 GPU session 4: GPU tests of the tree (k_audio LDS window, chain
# step in the reference's order), step-time A/B of the alpha-exact PLL words
# (c1a) and of k_rs on the front-end stream at <= 2048 channels (rsa)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/tests_r06d.log 2>&1
rc=$?; tail -4 $O/tests_r06d.log; [ $rc -le 1 ] || exit $rc
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 5 20 r05 cur c1a rsa > $O/ab2048_r06d.txt 2>&1 || exit 3
tail -4 $O/ab2048_r06d.txt
timeout -k 10 700 bash tools/gpu_abn.sh 5 20 r05 cur c1a c1x > $O/ab4096_r06d.txt 2>&1 || exit 3
tail -4 $O/ab4096_r06d.txt
