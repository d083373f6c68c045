#!/bin/bash
# GPU box: trainer tests + the trainer bench (launch-ahead, one-launch threshold A/B), phase stamps
# of the fused pre-split on MIXED, then the C2 trace + PMC passes (profile_gpu.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p $O
st() { echo "$1 rc=$2" >> $O/status.txt; [ $2 -eq 0 ] || exit $2; }
(cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "train or smoke or parity or long" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1); st pytest $?
(cd $R && SW_TRAIN_DEBUG=1 timeout -k 10 300 python -u tools/bench_train.py --workloads mixed128m,mixed128m,mixed128m --no-cpu > $O/train.jsonl 2> $O/train.err); st train $?
for fb in 64 256; do
  (cd $R && SW_TRAIN_FUSE_BLOCKS=$fb SW_TRAIN_DEBUG=1 timeout -k 10 300 python -u tools/bench_train.py --workloads mixed128m,mixed128m --no-cpu > $O/train_fb$fb.jsonl 2> $O/train_fb$fb.err); st train_fb$fb $?
done
(cd $R && SHREDWORD_HIP_LIB=$R/shredword_amd/libshredword_hip_stamps.so timeout -k 10 200 python3 tools/phase_stamps.py 250000 mixed fused > $O/stamps_fused.log 2>&1); st stamps $?
BENCH_ARGS="--config c5" timeout -k 10 600 bash $R/tools/gpu_ab_trace.sh ${TAG}_c5 libshredword_hip.so libshredword_hip_lpold.so > $O/ab_c5.log 2>&1; st ab_c5 $?
timeout -k 10 1100 bash $R/tools/profile_gpu.sh $TAG > $O/prof.log 2>&1; st prof $?
