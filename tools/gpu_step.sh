#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/t_on.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-kernel-timing > gpurun_out/t_off.json 2>/dev/null || true
python3 -c "
import json
a=json.load(open('gpurun_out/t_on.json'));print('timing on ', a['ms_per_step'], a['host_submit_ms'])
" ; python3 -c "
import json
b=json.loads(open('gpurun_out/t_off.json').read().strip().splitlines()[-1]);print('timing off', b['ms_per_step'], b['host_submit_ms'])
" || tail -5 gpurun_out/t_off.json
done
