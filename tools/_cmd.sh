set -o pipefail
L=libshredword_hip
bash tools/gpu_round.sh r3e pytest && bash tools/gpu_ab_trace.sh r3e_ab $L\_base.so $L\_rh2.so $L\_fz.so $L\_fz.so@--no-fused $L\_base.so@--config,c5 $L\_fz.so@--config,c5 $L\_base.so@--no-dedupe,--no-chunk-table $L\_fz.so@--no-dedupe,--no-chunk-table > gpurun_out/r3e_ab.txt 2>&1 && bash tools/gpu_round.sh r3e c2 gw1 trace_gw1
