#!/bin/bash
# Per-kernel unit counters for bench.py's "units" roofline (tools/unit_counters.py):
# four rocprofv3 --pmc passes on a short synchronized bench (each kernel alone),
# every pass within the gfx950 slot limits (SQ 8, TCC 4 with FETCH_SIZE = 3 and
# WRITE_SIZE = 2, GRBM 2) and under its own hard time limit.
# Usage (on the GPU box via gpurun): [UNITS_ARGS="--channels 2048"] tools/gpu_units.sh TAG
set -e
TAG=${1:-r05}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/units_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --sync-steps ${UNITS_ARGS:-} > "$OUT/bench_p$i.json" 2> "$OUT/p$i.err" || exit 1
done
CH=$(python3 -c "import json; print(json.load(open('$OUT/bench_p1.json'))['config']['channels_rank0'])")
python3 "$ROOT/tools/unit_counters.py" "$OUT" "$OUT/units.json" --channels "$CH" --block 4096 > /dev/null
python3 -c "import json; r=json.load(open('$OUT/units.json')); print(json.dumps({k: {n: round(v, 1) for n, v in e.items() if n != 'dispatches'} for k, e in r['kernels'].items()}))"
