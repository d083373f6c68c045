set -o pipefail
L=libshredword_hip
bash tools/gpu_round.sh r3f pytest gw1 trace_gw1 && bash tools/gpu_ab_trace.sh r3f_ab $L\_base.so $L\_wf1.so $L\_dw.so $L\_base.so $L\_dw.so $L\_base.so@--config,c5 $L\_dw.so@--config,c5 $L\_dw.so@--no-dedupe,--no-chunk-table > gpurun_out/r3f_ab.txt 2>&1
