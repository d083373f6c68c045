set -o pipefail
L=libshredword_hip
bash tools/gpu_round.sh r3i pytest && bash tools/gpu_ab_trace.sh r3i_ab $L\_base.so $L\_wf1.so $L\_lds.so $L\_base.so@--config,c5 $L\_wf1.so@--config,c5 $L\_lds.so@--config,c5 $L\_wf1.so@--no-dedupe,--no-chunk-table $L\_lds.so@--no-dedupe,--no-chunk-table > gpurun_out/r3i_ab.txt 2>&1
