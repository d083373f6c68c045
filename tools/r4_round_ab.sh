#!/bin/bash
# GPU box: -m gpu tests, then kernel-trace A/B of the fused-kernel variants (C2) and of the merge
# loop's pairing (entropy corpus; C2 with both memo shortcuts off)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out/abt_$TAG
(cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $R/gpurun_out/abt_$TAG/pytest.log 2>&1)
rc=$?; echo "pytest rc=$rc" >> $R/gpurun_out/abt_$TAG/status.txt; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_ab_trace.sh $TAG libshredword_hip_r4base.so libshredword_hip.so libshredword_hip_r1.so \
  libshredword_hip_r1w5.so libshredword_hip_r2w5.so \
  libshredword_hip.so@--corpus,entropy libshredword_hip_nopair.so@--corpus,entropy \
  libshredword_hip.so@--no-dedupe,--no-chunk-table libshredword_hip_nopair.so@--no-dedupe,--no-chunk-table
