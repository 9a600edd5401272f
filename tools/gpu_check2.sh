#!/bin/bash
# Round-2 check on the GPU box: full GPU parity suite (achieved errors logged),
# the old-sine A/B build on the oracle-compared tests, the default bench line,
# and a 2-rank gloo rehearsal of the multi-GPU bench on one GPU.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
L=$PWD/fmtuner-sdr_amd
rm -f gpurun_out/parity_*.jsonl
FMX_PARITY_LOG=gpurun_out/parity_new.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
if [ -f $L/libfmx_sinq.so ]; then
  FMX_LIB=$L/libfmx_sinq.so FMX_PARITY_LOG=gpurun_out/parity_sinq.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not smoke and not full_size_properties" > gpurun_out/gpu_tests_sinq.log 2>&1
  tail -2 gpurun_out/gpu_tests_sinq.log
fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
FMX_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { tail -30 gpurun_out/bench_gloo2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_gloo2.json'));print('gloo2', d['n_gpus'], d['value'], d['config'], d['scan'])"
