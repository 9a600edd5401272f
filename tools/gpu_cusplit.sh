#!/bin/bash
# Experiment: CU partitioning between the serial kernels (k_pll, k_rds) and
# the data-parallel ones (front end, audio) via stream CU masks.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/cu_$tag.json 2> gpurun_out/cu_$tag.err || { tail -5 gpurun_out/cu_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/cu_$tag.json'));print('$tag', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, d['check'])"
}
run base FMX_NONE=1
run s4 FMX_CU_SERIAL=4
run s8d FMX_CU_SERIAL=8,d
run s4d FMX_CU_SERIAL=4,d
run s8 FMX_CU_SERIAL=8
run s4all FMX_CU_SERIAL=4 FMX_CU_PAR_ALL=1
run s16d FMX_CU_SERIAL=16,d
