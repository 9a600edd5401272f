#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
L=$PWD/fmtuner-sdr_amd
STEREO=0 RDS_STAGE=0 FMX_DIAG_RDS_DUMP=1 FMX_LIB=$L/libfmx_pk2.so timeout -k 10 200 python tools/gpu_determinism.py 4096 8 1 > gpurun_out/det_pk2.log 2>&1; echo "pk2 dump rc=$? $(tail -1 gpurun_out/det_pk2.log)"
FMX_LIB=$L/libfmx_pk2.so FMX_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/iso_pk2.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/iso_pk2.json'));print('pk2 iso', {k:v['avg_ms'] for k,v in d['kernels'].items()})"
FMX_SERIAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/iso_cur.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/iso_cur.json'));print('cur iso', {k:v['avg_ms'] for k,v in d['kernels'].items()})"
exit 0
