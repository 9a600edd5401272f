#!/bin/bash
# round-6 GPU session 17: the RDS ring as checkpoints -- ring-refill tests,
# the RDS / reset parity suites, step-time A/B against HEAD~ (pre: ring
# written every call), k_rds bytes by request size
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
ROOT=$PWD
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rds_ring.py tests/test_gpu_parity.py tests/test_gpu_fe8_cold.py \
  tests/test_gpu_pipelined.py tests/test_gpu_determinism.py tests/test_gpu_cfg4_sizes.py -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/tests_r06q.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" $O/tests_r06q.log | tail -12; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 pre cur > $O/ab4096_r06q.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06q.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 pre cur > $O/ab2048_r06q.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06q.txt
P=$ROOT/$O/pmc_r06q
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
n=0
for cs in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  n=$((n + 1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d $P/p$n -o run \
    -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $P/bench_$n.json 2> $P/p$n.err || { echo "pass $n failed"; exit 3; }
done
python3 $ROOT/tools/pmc_reqsize.py $P/reqsize.json $P/p1 $P/p2 $P/p3
