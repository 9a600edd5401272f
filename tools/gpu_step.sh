#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log; grep -E "^U8" gpurun_out/gpu_tests.log | head -2 | cut -c1-200
bash tools/gpu_iso.sh 20 base cur
bash tools/gpu_abn.sh 3 100 base cur > gpurun_out/abn.log 2>&1; tail -2 gpurun_out/abn.log
FMX_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || { tail -20 gpurun_out/bench_g2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_g2.json'));print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['channels_rank0'], d['config']['total_channels'], d.get('scan',{}).get('points'))"
