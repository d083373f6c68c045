#!/bin/bash
# GPU box: kernel-trace A/B of library variants on C2 (and C5), then phase stamps of the fused kernel
# usage: tools/r4_ab2.sh TAG lib1 lib2 ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/abt_$TAG; mkdir -p $O
timeout -k 10 900 bash $R/tools/gpu_ab_trace.sh $TAG "$@" > $O/ab.txt 2>&1
rc=$?; echo "ab rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
if [ -f $R/shredword_amd/libshredword_hip_stamps.so ]; then
  (cd $R && SHREDWORD_HIP_LIB=$R/shredword_amd/libshredword_hip_stamps.so timeout -k 10 200 python3 tools/phase_stamps.py 250000 mixed fused > $O/stamps_fused.log 2>&1)
  rc=$?; echo "stamps rc=$rc" >> $O/status.txt
fi
