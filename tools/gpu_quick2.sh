#!/bin/bash
# GPU parity suite (stop at first failure) then the bench without the CPU
# leg, twice, plus one isolated (FMX_SERIAL=1) run for per-kernel times.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
rm -f gpurun_out/parity_new.jsonl
FMX_PARITY_LOG=gpurun_out/parity_new.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for t in a b; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/q_$t.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/q_$t.json'));print('$t', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
FMX_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/q_serial.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/q_serial.json'));print('serial', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
