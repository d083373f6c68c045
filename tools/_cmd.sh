set -o pipefail
L=libshredword_hip
bash tools/gpu_round.sh r3d pytest && bash tools/gpu_ab_trace.sh r3d_ab $L\_base.so $L\_cpf.so $L\_rh.so $L\_dd14.so $L\_ps.so $L\_wf.so $L\_base.so@--config,c5 $L\_wf.so@--config,c5 $L\_base.so@--no-dedupe,--no-chunk-table $L\_wf.so@--no-dedupe,--no-chunk-table > gpurun_out/r3d_ab.txt 2>&1 && bash tools/gpu_round.sh r3d gw1 trace_gw1
