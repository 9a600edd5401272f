#!/bin/bash
# Stage clocks (STAMPS variant library) pipelined + isolated, and bench A/B of
# the per-block RF level output.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
L=$PWD/fmtuner-sdr_amd
FMX_LIB=$L/libfmx_stamps.so timeout -k 10 120 python3 tools/fe_stamps.py > gpurun_out/stamps.txt 2>&1 || { tail gpurun_out/stamps.txt; exit 1; }
FMX_LIB=$L/libfmx_stamps.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > gpurun_out/stamps_serial.txt 2>&1 || exit 1
echo "== pipelined"; grep -v amdgpu.ids gpurun_out/stamps.txt
echo "== serial"; grep -v amdgpu.ids gpurun_out/stamps_serial.txt
for t in sig nosig sig2 nosig2; do
  extra=""; [[ $t == nosig* ]] && extra="--no-signal-level"
  timeout -k 10 200 python bench.py --no-cpu-baseline $extra > gpurun_out/ab_$t.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$t.json'));print('$t', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
FMX_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ab_serial.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/ab_serial.json'));print('serial', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
