#!/bin/bash
# GPU box: the e2e (PCIe-inclusive) leg at several pipeline run sizes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
for mb in "$@"; do
  (cd $R && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 3 --pipe-run-mb $mb > $O/e2e_$mb.log 2>&1)
  rc=$?; echo "e2e $mb rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
done
