#!/bin/bash
# GPU box: the pipelined host-path tests, then bench lines with the e2e (PCIe-inclusive) leg
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG; mkdir -p $O
(cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_c3_split.py -x -q --timeout 300 --timeout-method thread > $O/pytest_c3split.log 2>&1)
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
(cd $R && timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-steps 3 > $O/bench_c2_e2e.log 2>&1)
rc=$?; echo "bench rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
