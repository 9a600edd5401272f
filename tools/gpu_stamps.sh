#!/bin/bash
# Stage clocks of k_frontend / k_rds: builds a STAMPS=1 copy of libfmx in a
# scratch dir on the box (the in-tree library is left untouched).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/fe_stamps.py > gpurun_out/stamps.txt 2>&1
cat gpurun_out/stamps.txt
