#!/bin/bash
# round-6 final measurements, part 1 (final code): the whole GPU suite and smoke
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
bash tools/gpu_run.sh r06z tests smoke
