#!/bin/bash
# round-6 GPU session 11: k_rs with its schedule entries from L2 (no LDS
# staging) at 8 / 4 / 2 / 1 parts per channel group; the parity bisection
# across round 4's truncating-words commit (a4 = 600635d^, a5 = 600635d, r04)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipelined.py -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/tests_r06k.log 2>&1
rc=$?; tail -2 $O/tests_r06k.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 800 bash tools/gpu_abn.sh 4 20 r05 cur rs46 rs92 rs184 > $O/ab4096_r06k.txt 2>&1 || exit 3
tail -5 $O/ab4096_r06k.txt
FMX_AB_ARGS="--channels 2048" timeout -k 10 700 bash tools/gpu_abn.sh 4 20 r05 cur rs46 rs92 > $O/ab2048_r06k.txt 2>&1 || exit 3
tail -4 $O/ab2048_r06k.txt
B=$O/bisect2
mkdir -p $B
for v in a4 a5 r04 cur; do
  lib=$PWD/fmtuner-sdr_amd/libfmx_$v.so; [ $v = cur ] && lib=$PWD/fmtuner-sdr_amd/libfmx.so
  rm -f $B/parity_$v.jsonl
  FMX_LIB=$lib FMX_PARITY_LOG=$B/parity_$v.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "2m4 or 2m048 or cfg3_full or custom_deemph or weak_signal or staggered or cfg2" \
    > $B/tests_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $B/tests_$v.log)"; [ $rc -le 1 ] || exit $rc
done
python3 - <<'PY'
import json, statistics
for v in ["a4", "a5", "r04", "cur"]:
    try:
        d = [json.loads(l)["pcm_rms"] for l in open(f"gpurun_out/bisect2/parity_{v}.jsonl")]
    except OSError:
        print(v, "no log"); continue
    print(f"{v:4s} n={len(d)} pcm_rms median {statistics.median(d):.3e} max {max(d):.3e}")
PY
