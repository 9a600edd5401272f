#!/bin/bash
# Run-to-run spread of the pipelined bench at two step counts.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for steps in 20 20 20 100 100 100 400; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps $steps > gpurun_out/spread.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/spread.json'));print($steps, d['value'], d['ms_per_step'])"
done
