#!/bin/bash
# GPU box: the -m gpu tests on the default library, then kernel-trace A/B of library variants
# (tools/gpu_ab_trace.sh).  usage: tools/r4_ab.sh TAG [pytest|nopytest] spec...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
MODE=$1; shift
mkdir -p $R/gpurun_out/abt_$TAG
if [ "$MODE" = pytest ]; then
  (cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/abt_$TAG/pytest.log 2>&1)
  rc=$?; echo "pytest rc=$rc" >> $R/gpurun_out/abt_$TAG/status.txt; [ $rc -eq 0 ] || exit $rc
fi
bash $R/tools/gpu_ab_trace.sh $TAG "$@"
