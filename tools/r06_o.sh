#!/bin/bash
# round-6 GPU session 15: intermediate rows padded off the 1-KB grid
# (Handle::row, FMX_ROW_PAD=0 the unpadded A/B arm) -- parity suites,
# k_rds taps in registers (hreg2), serial waves at priority 3 (prio3), step-time A/B at 4096 / 2048 channels, HBM bytes by request size per arm
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
ROOT=$PWD
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipelined.py tests/test_gpu_cfg4_sizes.py \
  tests/test_facades.py tests/test_gpu_fe8_cold.py -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_r06o.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_r06o.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur nopad:FMX_ROW_PAD=0 hreg2 prio3 > $O/ab4096_r06o.txt 2>&1 || exit 3
tail -4 $O/ab4096_r06o.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur nopad:FMX_ROW_PAD=0 hreg2 prio3 > $O/ab2048_r06o.txt 2>&1 || exit 3
tail -4 $O/ab2048_r06o.txt
cd /tmp && export TMPDIR=/tmp
for arm in pad nopad; do
  P=$ROOT/$O/pmc_r06o_$arm
  mkdir -p $P
  export FMX_ROW_PAD=1; [ $arm = nopad ] && export FMX_ROW_PAD=0
  n=0
  for cs in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    n=$((n + 1))
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d $P/p$n -o run \
      -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $P/bench_$n.json 2> $P/p$n.err || { echo "pass $n failed"; exit 3; }
  done
  echo "== $arm"; python3 $ROOT/tools/pmc_reqsize.py $P/reqsize.json $P/p1 $P/p2 $P/p3
done
