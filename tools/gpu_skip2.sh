#!/bin/bash
# Diagnostic: pipelined step time with kernels left out (FMX_DIAG_SKIP), each twice.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for skip in none rds pll audio rds,pll rds,pll,audio none; do
  FMX_DIAG_SKIP=$skip timeout -k 10 120 python bench.py --no-cpu-baseline --steps 60 > gpurun_out/skip_$skip.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/skip_$skip.json'));print('$skip', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
