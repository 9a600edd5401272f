#!/bin/bash
# Interleaved A/B of library variants: tools/gpu_abn.sh REPS STEPS name1 name2 ...
# (name "cur" = libfmx.so, "name:VAR=VAL" = libfmx.so with that environment,
# else fmtuner-sdr_amd/libfmx_<name>.so); prints the per-run ms/step and the
# median per variant.  FMX_AB_ARGS adds bench.py arguments (e.g. "--channels 2048").
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
REPS=$1; STEPS=$2; shift 2
L=$PWD/fmtuner-sdr_amd
for r in $(seq 1 $REPS); do
  for v in "$@"; do
    lib=$L/libfmx.so; envv=FMX_AB_NONE=1; name=$v
    case "$v" in
      *:*) name=${v%%:*}; envv=${v#*:} ;;
      cur) ;;
      *) lib=$L/libfmx_$v.so ;;
    esac
    env "$envv" FMX_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps $STEPS $FMX_AB_ARGS > gpurun_out/abn_${name}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abn_${name}_$r.json'));print('$name', $r, d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
  done
done | tee gpurun_out/abn.txt
python3 - "$@" <<'PY'
import sys, statistics
rows = [l.split() for l in open('gpurun_out/abn.txt')]
for v in (a.split(':')[0] for a in sys.argv[1:]):
    xs = sorted(float(r[2]) for r in rows if r[0] == v)
    print(f"{v:10s} median {statistics.median(xs):.4f}  min {xs[0]:.4f}  max {xs[-1]:.4f}  n={len(xs)}")
PY
