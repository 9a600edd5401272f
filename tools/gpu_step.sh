#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
FMX_DIAG_HOST=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/hd.json 2> gpurun_out/hd.err
grep "fmx host" gpurun_out/hd.err; python3 -c "import json;d=json.load(open('gpurun_out/hd.json'));print(d['ms_per_step'], d['host_submit_ms'])"
