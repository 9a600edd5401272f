#!/bin/bash
# scratch GPU step 2 (edited per experiment)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
bash tools/gpu_abn.sh 3 100 base cur > gpurun_out/abn.log 2>&1; tail -3 gpurun_out/abn.log
python3 -c "
import json
for v in ('base','cur'):
    d=json.load(open('gpurun_out/abn_%s_1.json'%v)); print(v, d.get('host_submit_ms'), d['ms_per_step'])"
