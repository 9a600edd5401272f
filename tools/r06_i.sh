#!/bin/bash
# round-6 GPU session 9: where round 5's PCM error growth came from -- the
# same parity tests (with FMX_PARITY_LOG) on libraries of round 4's end (r04),
# round 5's first commit (p0), the PLL chain change (p1), the per-channel cold
# start (p2), round 5's end (r05) and the current tree (cur)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out/bisect
mkdir -p $O
for v in r04 p0 p1 p2 r05 cur; do
  lib=$PWD/fmtuner-sdr_amd/libfmx_$v.so; [ $v = cur ] && lib=$PWD/fmtuner-sdr_amd/libfmx.so
  rm -f $O/parity_$v.jsonl
  FMX_LIB=$lib FMX_PARITY_LOG=$O/parity_$v.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "2m4 or 2m048 or cfg3_full or custom_deemph or weak_signal or staggered or cfg2" \
    > $O/tests_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $O/tests_$v.log)"; [ $rc -le 1 ] || exit $rc
done
python3 - <<'PY'
import json, statistics
O = "gpurun_out/bisect"
base = {}
for v in ["r04", "p0", "p1", "p2", "r05", "cur"]:
    try:
        recs = [json.loads(l) for l in open(f"{O}/parity_{v}.jsonl")]
    except OSError:
        print(v, "no log"); continue
    d = {(r["test"], r["channel"]): r["pcm_rms"] for r in recs}
    if not base: base = d
    shared = [d[k] / base[k] for k in d if k in base and base[k] > 0]
    print(f"{v:4s} n={len(d)} pcm_rms median {statistics.median(d.values()):.3e} max {max(d.values()):.3e}  "
          f"median ratio to r04 {statistics.median(shared) if shared else float('nan'):.3f}")
PY
