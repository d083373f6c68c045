#!/bin/bash
# GPU box: the gpu tests, then an A/B kernel trace of library variants (tools/gpu_ab_trace.sh)
# usage: tools/gpu_test_ab.sh TAG lib1.so lib2.so ...
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_ab_trace.sh "$@"
