#!/bin/bash
# round-6 final measurements, part 2 (final code): unit counters at 4096 and
# 2048 channels (into profiles/ on the box, so that the bench lines carry
# them), the default bench with the CPU baseline, the driver-shaped 20-step
# bench, rocprofv3 kernel stats of that shape, the channel sweep
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
O=gpurun_out
bash tools/gpu_run.sh r06z units || exit 3
cp $O/units_r06z/units.json profiles/r06z_units.json && cp $O/units_r06z_2048/units.json profiles/r06z_2048_units.json || exit 3
bash tools/gpu_run.sh r06z benchfull bench stats sweep
