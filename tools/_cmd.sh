set -o pipefail
L=libshredword_hip
bash tools/gpu_ab_trace.sh r3j_ab $L\_lds.so $L\_pf1.so $L\_pf2.so $L\_lds.so@--no-dedupe,--no-chunk-table $L\_pf1.so@--no-dedupe,--no-chunk-table $L\_pf2.so@--no-dedupe,--no-chunk-table $L\_nm.so@--no-dedupe,--no-chunk-table $L\_nm.so $L\_nm.so@--config,c5 $L\_lds.so@--config,c5 $L\_pf2.so@--config,c5 > gpurun_out/r3j_ab.txt 2>&1
