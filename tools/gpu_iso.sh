#!/bin/bash
# Isolated per-kernel times (FMX_SERIAL=1: every kernel on one stream) of
# library variants: tools/gpu_iso.sh STEPS name1 name2 ... (names as gpu_abn.sh;
# a trailing "+nosig" runs the bench with --no-signal-level)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
STEPS=$1; shift
L=$PWD/fmtuner-sdr_amd
for v in "$@"; do
  extra=""; vv=$v
  case "$v" in *+nosig) extra="--no-signal-level"; vv=${v%+nosig} ;; esac
  lib=$L/libfmx.so; envv=FMX_AB_NONE=1; name=$vv
  case "$vv" in
    *:*) name=${vv%%:*}; envv=${vv#*:} ;;
    cur) ;;
    *) lib=$L/libfmx_$vv.so ;;
  esac
  env "$envv" FMX_SERIAL=1 FMX_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps $STEPS $extra > gpurun_out/iso_$name.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/iso_$name.json'));print('$v', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
