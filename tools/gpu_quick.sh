set -u
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q.log 2>&1 || exit 1
SHREDWORD_HIP_LIB=$PWD/shredword_amd/libshredword_hip_stamps.so timeout -k 10 200 python tools/phase_stamps.py > gpurun_out/stamps.log 2>&1
