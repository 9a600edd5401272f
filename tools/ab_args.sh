#!/bin/bash
# Interleaved A/B of bench.py argument sets on one library:
#   tools/ab_args.sh REPS STEPS "args A" "args B" ...   (arm "-" = no extra arguments)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
REPS=$1; STEPS=$2; shift 2
for r in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    i=$((i + 1)); A=$v; [ "$A" = "-" ] && A=""
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps $STEPS $A > gpurun_out/aba_${i}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/aba_${i}_$r.json'));print('arm$i', $r, d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
  done
done | tee gpurun_out/aba.txt
python3 - "$@" <<'PY'
import sys, statistics
rows = [l.split() for l in open('gpurun_out/aba.txt')]
for i, a in enumerate(sys.argv[1:], 1):
    xs = sorted(float(r[2]) for r in rows if r[0] == f"arm{i}")
    print(f"arm{i} [{a}] median {statistics.median(xs):.4f}  min {xs[0]:.4f}  max {xs[-1]:.4f}  n={len(xs)}")
PY
