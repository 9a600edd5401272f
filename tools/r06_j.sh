#!/bin/bash
# round-6 GPU session 10: RDS stream behind k_pilot (rap) A/B; round-5 parity
# bisection (tools/r06_i.sh); HBM bytes per kernel by request size (three
# counter passes, tools/pmc_reqsize.py)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
ROOT=$PWD
O=gpurun_out
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur rap > $O/ab4096_r06j.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06j.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur rap > $O/ab2048_r06j.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06j.txt
bash tools/r06_i.sh || exit 3
P=$ROOT/$O/pmc_r06j
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
n=0
for cs in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  n=$((n + 1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d $P/p$n -o run \
    -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $P/bench_$n.json 2> $P/p$n.err || { echo "pass $n failed"; exit 3; }
done
python3 $ROOT/tools/pmc_reqsize.py $P/reqsize.json $P/p1 $P/p2 $P/p3
