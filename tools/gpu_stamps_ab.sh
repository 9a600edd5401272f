#!/bin/bash
# k_rds / k_pll stage clocks of STAMPS builds given as FMX_LIB names (libfmx_st_<tag>.so), isolated streams.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
L=$PWD/fmtuner-sdr_amd
for v in ${ST_TAGS:-old new}; do
  echo "=== $v serial"; FMX_LIB=$L/libfmx_st_$v.so FMX_SERIAL=1 timeout -k 10 120 python3 tools/fe_stamps.py 2>&1 | grep -v amdgpu.ids | sed -n '/k_pll/,$p' || exit 1
done
