#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG; mkdir -p $O
(cd $R && SW_PIPE_TRACE=${SW_PIPE_TRACE:-} timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 3 > $O/bench_c2_e2e.log 2>&1)
rc=$?; echo "bench rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
