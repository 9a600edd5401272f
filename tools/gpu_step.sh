#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
bash tools/gpu_prof2.sh r02g > gpurun_out/prof2_r02g.log 2>&1 || { tail -20 gpurun_out/prof2_r02g.log; exit 1; }
timeout -k 10 300 python bench.py --pmc-json gpurun_out/prof_r02g/pmc_frontend.json > gpurun_out/bench_r02g.json 2> gpurun_out/bench_r02g.err
timeout -k 10 300 python bench.py --no-cpu-baseline --pmc-json gpurun_out/prof_r02g/pmc_frontend.json > gpurun_out/bench_r02g_repeat.json 2>> gpurun_out/bench_r02g.err
python3 -c "
import json
for f in ('bench_r02g','bench_r02g_repeat'):
    d=json.load(open('gpurun_out/%s.json'%f)); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['valu_path']['frac'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
