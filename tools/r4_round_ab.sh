#!/bin/bash
# GPU box: -m gpu tests, the trainer with / without the merge launched ahead (mixed128m, digests
# compared), then kernel-trace A/B of the fused-kernel variants (C2) and of the merge loop's
# pairing (entropy corpus; C2 with both memo shortcuts off)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/abt_$TAG
mkdir -p $O
(cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1)
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
(cd $R && SW_TRAIN_DEBUG=1 timeout -k 10 300 python -u tools/bench_train.py --workloads mixed128m,mixed128m --no-cpu > $O/train_ahead.jsonl 2> $O/train_ahead.err)
rc=$?; echo "train ahead rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
(cd $R && SW_TRAIN_DEBUG=1 SW_TRAIN_NO_AHEAD=1 timeout -k 10 300 python -u tools/bench_train.py --workloads mixed128m --no-cpu > $O/train_noahead.jsonl 2> $O/train_noahead.err)
rc=$?; echo "train noahead rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_ab_trace.sh $TAG libshredword_hip_r4base.so libshredword_hip.so libshredword_hip_r1.so \
  libshredword_hip_r1w5.so libshredword_hip_r2w5.so \
  libshredword_hip.so@--corpus,entropy libshredword_hip_nopair.so@--corpus,entropy \
  libshredword_hip.so@--no-dedupe,--no-chunk-table libshredword_hip_nopair.so@--no-dedupe,--no-chunk-table
