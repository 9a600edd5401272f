#!/bin/bash
# round-6 GPU session 20: the decimator's tap window twice in LDS (odd-g
# lanes read a copy 12 dwords along the banks: no 2-way fragment conflicts)
# -- front-end parity suites on that library, bank-conflict counters,
# step-time A/B at 4096 / 2048 channels
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
ROOT=$PWD
O=gpurun_out
FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_qc.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fe8_cold.py \
  tests/test_gpu_pipelined.py tests/test_gpu_determinism.py tests/test_gpu_weak_carrier.py -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "not graft_smoke" > $O/tests_r06s.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests_r06s.log | tail -6; [ $rc -le 1 ] || exit $rc
P=$ROOT/$O/cnt_r06s
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for v in cur qc; do
  L=$ROOT/fmtuner-sdr_amd/libfmx.so; [ $v = qc ] && L=$ROOT/fmtuner-sdr_amd/libfmx_qc.so
  FMX_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv \
    -d $P/$v -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sync-steps > $P/bench_$v.json 2> $P/$v.err || exit 3
done
cd $ROOT
python3 - <<'PY'
import csv, glob, collections
for v in ("cur", "qc"):
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/cnt_r06s/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_fe8" in r["Kernel_Name"]:
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x) / 1e6, 2) for k, x in d.items()})
PY
timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur qc > $O/ab4096_r06s.txt 2>&1 || exit 3
tail -2 $O/ab4096_r06s.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 cur qc > $O/ab2048_r06s.txt 2>&1 || exit 3
tail -2 $O/ab2048_r06s.txt
