#!/bin/bash
# VALU instruction mix per kernel (two SQ counter passes, steps synchronized):
# where the front end's issue slots go.  Usage: tools/gpu_valu_mix.sh TAG
set -e
TAG=${1:-mix}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/mix_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VALU_FLOPS_FP32"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --sync-steps > "$OUT/bench_p$i.json" 2> "$OUT/p$i.err" || exit 1
done
python3 "$ROOT/tools/counter_summary.py" "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
