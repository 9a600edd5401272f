#!/bin/bash
# SQ counter passes on the 1-GPU bench (steps synchronized so the frontend
# runs alone).  Usage (on the GPU box via gpurun): [CNT_ARGS="--channels 2048"] tools/gpu_counters.sh TAG
set -e
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/cnt_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --sync-steps ${CNT_ARGS:-} > "$OUT/bench_p$i.json" 2> "$OUT/p$i.err" || exit 1
done
python3 "$ROOT/tools/counter_summary.py" "$OUT" > "$OUT/summary.txt"
