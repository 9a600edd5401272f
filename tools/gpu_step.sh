#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
bash tools/gpu_profile.sh r02i 10 > gpurun_out/profile_r02i.log 2>&1 || { tail -20 gpurun_out/profile_r02i.log; exit 1; }
timeout -k 10 300 python bench.py --pmc-json gpurun_out/prof_r02i/pmc_frontend.json > gpurun_out/bench_r02i.json 2> gpurun_out/bench_r02i.err
python3 -c "import json;d=json.load(open('gpurun_out/bench_r02i.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['valu_path']['frac'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
