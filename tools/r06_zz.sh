#!/bin/bash
# round-6 final measurements, re-taken once after the last kernel-placement
# change (k_rs part sizes below 4096 channels): GPU suite, smoke, unit
# counters (into profiles/ on the box for the bench lines), default bench,
# 20-step bench, kernel stats, channel sweep
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
bash tools/gpu_run.sh r06zz tests smoke units || exit 3
cp $O/units_r06zz/units.json profiles/r06zz_units.json && cp $O/units_r06zz_2048/units.json profiles/r06zz_2048_units.json || exit 3
bash tools/gpu_run.sh r06zz benchfull bench stats sweep
