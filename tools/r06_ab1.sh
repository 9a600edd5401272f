bash tools/pll_forms_ab.sh cur c1 c2 c3 c3w c1w > gpurun_out/pllab_summary.txt 2>&1 && cat gpurun_out/pllab_summary.txt && \
FMX_AB_ARGS="--channels 2048" timeout -k 10 500 bash tools/gpu_abn.sh 3 20 cur c1 c2 c3 c3w c1w > gpurun_out/pllab_ab2048.txt 2>&1 && tail -6 gpurun_out/pllab_ab2048.txt && \
timeout -k 10 500 bash tools/gpu_abn.sh 3 20 cur c1 c2 c3 c3w c1w > gpurun_out/pllab_ab4096.txt 2>&1 && tail -6 gpurun_out/pllab_ab4096.txt
