#!/bin/bash
# round-6 GPU session 8: the fusion bound -- the pipelined step with k_rs
# skipped (diagnostics library, outputs wrong, timing only) against the full
# step, at 2048 and 4096 channels; k_pilot skipped likewise; the TCC counters
# this rocprofv3 offers (for the request-size calibration of FETCH_SIZE)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
ROOT=$PWD
O=gpurun_out
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $ROOT/$O/list_avail.txt 2>&1); grep -o "TCC_EA0_[A-Za-z0-9_]*" $O/list_avail.txt | sort -u | tr '\n' ' '; echo
D=$PWD/fmtuner-sdr_amd/libfmx_diag.so
for C in 2048 4096; do
  for r in 1 2 3 4; do
    for sk in none krs pilot; do
      FMX_DIAG_SKIP=$sk FMX_LIB=$D timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --channels $C \
        > $O/skip_${sk}_${C}_$r.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.load(open('$O/skip_${sk}_${C}_$r.json'));print('$sk', $C, $r, d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
    done
  done
done | tee $O/skip_r06h.txt
python3 - <<'PY'
import statistics
rows = [l.split() for l in open('gpurun_out/skip_r06h.txt')]
for C in ('2048', '4096'):
    for sk in ('none', 'krs', 'pilot'):
        xs = sorted(float(r[3]) for r in rows if r[0] == sk and r[1] == C)
        print(C, sk, 'median %.4f' % statistics.median(xs), 'n=%d' % len(xs))
PY
