#!/bin/bash
# round-6 GPU session 6: GPU suite (tap windows by LDS-DMA), stage clocks,
# step-time A/B against round 5's library at 2048 / 4096 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/tests_r06f.log 2>&1
rc=$?; tail -3 $O/tests_r06f.log; [ $rc -le 1 ] || exit $rc
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_serial_r06f.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/stamps_serial_r06f.txt | head -12
DECIM=1 FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag_dec.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_dec_serial_r06f.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/stamps_dec_serial_r06f.txt | head -12
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 5 20 r05 cur > $O/ab2048_r06f.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06f.txt
timeout -k 10 700 bash tools/gpu_abn.sh 5 20 r05 cur > $O/ab4096_r06f.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06f.txt
