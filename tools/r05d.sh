set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_r05f.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/tests_r05f.log | head -5 | cut -c1-200; tail -3 $O/tests_r05f.log
[ $rc -le 1 ] || exit $rc
for rep in 1 2 3; do
  for arm in off on; do
    X=""; [ $arm = on ] && X="--retune-per-step"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $X > $O/ab_r05f_${arm}_$rep.json 2> $O/ab_r05f_${arm}_$rep.err || exit 1
    python3 -c "import json; r=json.load(open('$O/ab_r05f_${arm}_$rep.json')); print('$arm', r['ms_per_step'], {k: (v['avg_ms'], v['launches']) for k, v in r['kernels'].items()})"
  done
done
