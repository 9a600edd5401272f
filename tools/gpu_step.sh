#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
FMX_DIAG_HOST=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/hd.json 2> gpurun_out/hd.err
grep "fmx host" gpurun_out/hd.err; python3 -c "import json;d=json.load(open('gpurun_out/hd.json'));print(d['ms_per_step'], d['host_submit_ms'])"
bash tools/gpu_step2.sh
