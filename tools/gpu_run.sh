#!/bin/bash
# One GPU-box session of round-3 work: steps chosen by name, each under its
# own time limit; a step that faults, aborts or times out ends the session
# (no further GPU step runs).  Test failures (pytest rc 1) do not.
#   tools/gpu_run.sh TAG step [step ...]
# steps: tests (pytest -m gpu), ptests (pipelined parity only), smoke,
#        bench (driver-shaped: --steps 20 --warmup 5), benchfull (default
#        bench with the CPU baseline), trace (rocprofv3 kernel trace + gaps),
#        stats (rocprofv3 --kernel-trace --stats), pmc (FETCH / WRITE passes),
#        ubench (tools/ubench/chainlat), sweep (channel sweep), stamps (stage clocks,
#        diagnostics library), iso (isolated kernel times, diagnostics library),
#        units (unit counters for bench.py's roofline), retune_ab (a retune per step vs none)
TAG=$1
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
O=gpurun_out
mkdir -p $O
fatal() { # rc of a GPU step: 0 ok, 1 test failures; anything else ends the session
  case "$1" in
    0|1) return 1 ;;
    *) echo "step $2: rc $1 -- stopping"; return 0 ;;
  esac
}
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $O/tests_$TAG.log 2>&1; rc=$?
      tail -3 $O/tests_$TAG.log ;;
    ptests)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_determinism.py -x -v --timeout 300 \
        --timeout-method thread -p no:cacheprovider > $O/ptests_$TAG.log 2>&1; rc=$?
      tail -3 $O/ptests_$TAG.log ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1; rc=$?
      tail -1 $O/smoke_$TAG.log ;;
    bench)
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err; rc=$?
      python3 -c "import json,sys; r=json.load(open('$O/bench_$TAG.json')); print(r['value'], r['ms_per_step'], {k: v['avg_ms'] for k, v in r['kernels'].items()}, r['host_submit_ms'])" ;;
    benchfull)
      timeout -k 10 400 python bench.py > $O/benchfull_$TAG.json 2> $O/benchfull_$TAG.err; rc=$?
      python3 -c "import json,sys; r=json.load(open('$O/benchfull_$TAG.json')); print(r['value'], r['ms_per_step'], r['cpu_baseline']['value'] if r['cpu_baseline'] else None)" ;;
    trace)
      bash tools/gpu_trace.sh trace_$TAG > $O/trace_$TAG.log 2>&1; rc=$?
      head -30 $O/trace_$TAG.log ;;
    stats)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/stats_$TAG" -o run \
        -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline ${FMX_AB_ARGS:-} > "$ROOT/$O/stats_${TAG}_bench.json" 2> "$ROOT/$O/stats_$TAG.err"); rc=$?
      cat $O/stats_$TAG/*kernel_stats.csv 2>/dev/null | cut -c1-160 | head -8 ;;
    pmc)
      bash tools/gpu_profile_pmc.sh "$TAG" > $O/pmc_$TAG.log 2>&1; rc=$?
      tail -12 $O/pmc_$TAG.log ;;
    skips)
      # pipelined step with kernels left out (diagnostics library, FMX_DIAG_SKIP):
      # what each co-runner costs the front end's live time
      for sk in none pll rds audio pll,rds,audio; do
        FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so FMX_DIAG_SKIP=$sk timeout -k 10 200 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline > $O/skip_${sk}_$TAG.json 2> $O/skip_${sk}_$TAG.err || { rc=$?; break; }
        python3 -c "import json,sys; r=json.load(open('$O/skip_${sk}_$TAG.json')); print('skip $sk', r['ms_per_step'], {k: v['avg_ms'] for k, v in r['kernels'].items()})"
        rc=0
      done ;;
    counters)
      # SQ counter passes (tools/gpu_counters.sh): instruction mix / waits per kernel
      bash tools/gpu_counters.sh $TAG > $O/counters_$TAG.log 2>&1; rc=$?
      cat $O/cnt_$TAG/summary.txt 2>/dev/null | head -80 ;;
    ubench)
      timeout -k 10 120 tools/ubench/chainlat > $O/chainlat_$TAG.txt 2>&1; rc=$?
      cat $O/chainlat_$TAG.txt ;;
    stamps)
      # diagnostics library: stage clocks, pipelined and then isolated (one stream)
      FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_$TAG.txt 2>&1 && \
      FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_serial_$TAG.txt 2>&1; rc=$?
      grep -v amdgpu.ids $O/stamps_$TAG.txt; echo "-- serial"; grep -v amdgpu.ids $O/stamps_serial_$TAG.txt ;;
    stamps:*)
      # stage clocks of another diagnostics library: stamps:diag_dec (decimator split), stamps:diag_t8
      V=${step#stamps:}
      EX=""
      case $V in *dec*) EX="DECIM=1" ;; esac
      case $V in *t8*) EX="$EX PLL_CH=32" ;; esac
      env $EX FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_$V.so timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_${V}_$TAG.txt 2>&1 && \
      env $EX FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_$V.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py > $O/stamps_serial_${V}_$TAG.txt 2>&1; rc=$?
      grep -v amdgpu.ids $O/stamps_${V}_$TAG.txt; echo "-- serial"; grep -v amdgpu.ids $O/stamps_serial_${V}_$TAG.txt ;;
    iso)
      # isolated per-kernel times (diagnostics library, one stream)
      FMX_LIB=$PWD/fmtuner-sdr_amd/libfmx_diag.so FMX_SERIAL=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/iso_$TAG.json 2> $O/iso_$TAG.err; rc=$?
      python3 -c "import json,sys; r=json.load(open('$O/iso_$TAG.json')); print('isolated', r['ms_per_step'], {k: v['avg_ms'] for k, v in r['kernels'].items()})" ;;
    ab:*)
      # interleaved A/B of library variants: ab:cur,t16,t4 (tools/gpu_abn.sh, 3 reps x 20 steps)
      timeout -k 10 900 bash tools/gpu_abn.sh 3 20 $(echo ${step#ab:} | tr ',' ' ') > $O/ab_$TAG.log 2>&1; rc=$?
      tail -6 $O/ab_$TAG.log ;;
    sweep)
      bash tools/gpu_sweep.sh $TAG > $O/sweep_$TAG.log 2>&1; rc=$?
      cat $O/sweep_$TAG.log ;;
    units)
      # per-kernel unit counters (VALU / MFMA / LDS / HBM) for bench.py's roofline units
      bash tools/gpu_units.sh $TAG > $O/units_$TAG.log 2>&1 && \
      UNITS_ARGS="--channels 2048" bash tools/gpu_units.sh ${TAG}_2048 >> $O/units_$TAG.log 2>&1; rc=$?
      cat $O/units_$TAG.log ;;
    retune_ab)
      # a retune of one channel before every step against none, interleaved, 3 x 20 steps each
      rc=0
      for rep in 1 2 3; do
        for arm in off on; do
          X=""; [ $arm = on ] && X="--retune-per-step"
          timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $X > $O/retune_${TAG}_${arm}_$rep.json \
            2> $O/retune_${TAG}_${arm}_$rep.err || { rc=$?; break 2; }
          python3 -c "import json; r=json.load(open('$O/retune_${TAG}_${arm}_$rep.json')); print('$arm', r['ms_per_step'], {k: (v['avg_ms'], v['launches']) for k, v in r['kernels'].items()})"
        done
      done ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== $step rc=$rc $(date +%T)"
  if fatal $rc $step; then exit $rc; fi
done
exit 0
