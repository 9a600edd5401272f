set -e
D=$PWD/fmtuner-sdr_amd/libfmx_diag.so
FMX_LIB=$D bash tools/gpu_trace.sh tr_diag > gpurun_out/tr_diag.log 2>&1
FMX_LIB=$D FMX_DIAG_NOWAIT=1 bash tools/gpu_trace.sh tr_nowait > gpurun_out/tr_nowait.log 2>&1
FMX_LIB=$D FMX_DIAG_SAPRIO=1 bash tools/gpu_trace.sh tr_saprio > gpurun_out/tr_saprio.log 2>&1
FMX_LIB=$D FMX_DIAG_SKIP=audio bash tools/gpu_trace.sh tr_noaudio > gpurun_out/tr_noaudio.log 2>&1
FMX_LIB=$D FMX_DIAG_SKIP=rds bash tools/gpu_trace.sh tr_nords > gpurun_out/tr_nords.log 2>&1
