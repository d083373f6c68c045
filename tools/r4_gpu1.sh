#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4a; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/bench_fused.log 2>&1; rc=$?; echo "bench_fused rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --e2e-steps 0 --no-fused > $O/bench_unfused.log 2>&1; rc=$?; echo "bench_unfused rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc" >> $O/status.txt
exit $rc
