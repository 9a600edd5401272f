#!/bin/bash
# Diagnostic: pipelined step time with kernels left out (FMX_DIAG_SKIP).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for skip in none rds pll rds,pll rds,pll,audio; do
  FMX_DIAG_SKIP=$skip timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/skip_$skip.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/skip_$skip.json'));print('$skip', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
