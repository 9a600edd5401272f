#!/bin/bash
# round-6 GPU session 5: the shipped PLL forms' exhaustive sweep (new golden),
# the GPU suite with parity logging, k_fe8 / k_rds / k_pll stage clocks of
# the current code (diagnostics library), and a rocprof kernel-stats run
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
FMX_PLLMATH_OUT=$O/pllmath_r06e.json timeout -k 10 200 python -u -m pytest tests/test_gpu_pllmath.py -q -p no:cacheprovider \
  --timeout 150 --timeout-method thread > $O/pllmath_r06e.log 2>&1
rc=$?; tail -3 $O/pllmath_r06e.log; cat $O/pllmath_r06e.json; [ $rc -le 1 ] || exit $rc
rm -f $O/parity_r06e.jsonl
FMX_PARITY_LOG=$O/parity_r06e.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/tests_r06e.log 2>&1
rc=$?; tail -4 $O/tests_r06e.log; [ $rc -le 1 ] || exit $rc
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_r06e.txt 2>&1 || exit 3
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_serial_r06e.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/stamps_r06e.txt; echo "-- serial"; grep -v amdgpu.ids $O/stamps_serial_r06e.txt
bash tools/gpu_run.sh r06e stats
