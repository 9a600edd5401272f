#!/bin/bash
# Round-6 A/B of the stereo PLL's arithmetic forms (fmx_math.h: FMX_PLL_CHAIN,
# FMX_WORD_SINCOS, FMX_PLL_WORDS).  Per variant V (cur = libfmx.so, else
# fmtuner-sdr_amd/libfmx_V.so with tests/hip/libpllmath_V.so):
#   * the exhaustive sweep of its chain arithmetic -> gpurun_out/pllab/pllmath_V.json
#     (the test's golden comparison fails for the non-shipped forms: expected)
#   * the GPU parity suites with FMX_PARITY_LOG -> gpurun_out/pllab/parity_V.jsonl
# Usage: tools/pll_forms_ab.sh V [V ...]
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out/pllab
mkdir -p $O
for v in "$@"; do
  lib=$PWD/fmtuner-sdr_amd/libfmx_$v.so; plib=$PWD/tests/hip/libpllmath_$v.so
  [ "$v" = cur ] && { lib=$PWD/fmtuner-sdr_amd/libfmx.so; plib=$PWD/tests/hip/libpllmath.so; }
  rm -f $O/parity_$v.jsonl
  FMX_PLLMATH_LIB=$plib FMX_PLLMATH_OUT=$O/pllmath_$v.json timeout -k 10 120 python -u -m pytest \
    tests/test_gpu_pllmath.py -q -x -p no:cacheprovider --timeout 100 --timeout-method thread > $O/pllmath_$v.log 2>&1
  rc=$?
  case $rc in 0|1) ;; *) echo "$v pllmath rc $rc -- stopping"; exit $rc ;; esac
  FMX_LIB=$lib FMX_PARITY_LOG=$O/parity_$v.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_pipelined.py tests/test_gpu_cfg4_sizes.py tests/test_gpu_weak_carrier.py -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?
  echo "$v tests rc $rc: $(tail -1 $O/tests_$v.log)"
  case $rc in 0|1) ;; *) echo "$v tests rc $rc -- stopping"; exit $rc ;; esac
done
python3 - "$@" <<'PY'
import json, sys, statistics
O = "gpurun_out/pllab"
for v in sys.argv[1:]:
    try:
        recs = [json.loads(l) for l in open(f"{O}/parity_{v}.jsonl")]
    except OSError:
        print(v, "no parity log"); continue
    pr = [r["pcm_rms"] for r in recs if "pcm_rms" in r]
    pm = [r["pcm_max"] for r in recs if "pcm_max" in r]
    try:
        pl = json.load(open(f"{O}/pllmath_{v}.json"))
        pb = pl.get("chain_phase_bias"); cs = pl.get("chain_sin_vs_ref_phase")
    except OSError:
        pb = cs = None
    print(f"{v:5s} n={len(pr)} pcm_rms median {statistics.median(pr):.3e} max {max(pr):.3e}  "
          f"pcm_max max {max(pm):.3e}  chain_sin_vs_ref {cs}  phase_bias {pb}")
PY
