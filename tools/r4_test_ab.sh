#!/bin/bash
# GPU box: the whole -m gpu suite, then a kernel-trace A/B (tools/r4_ab2.sh) of the given specs
# usage: tools/r4_test_ab.sh TAG spec...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/abt_$TAG; mkdir -p $O
(cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1)
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
[ $# -gt 0 ] && BENCH_ARGS="--steps 20" bash $R/tools/r4_ab2.sh $TAG "$@"
exit 0
