#!/bin/bash
# GPU box: the whole -m gpu suite, then the round-4 bench lines (tools/r4_final.sh steps)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
(cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1)
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
bash $R/tools/r4_final.sh $TAG "$@"
