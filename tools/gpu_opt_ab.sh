#!/bin/bash
# Device-rate A/B of bench options (GPU box): each argument is one variant's bench flags, run
# twice, interleaved.  usage: tools/gpu_opt_ab.sh "" "--no-merge-streams" "--config c5" ...
set -u
OUT=gpurun_out/opt_ab; mkdir -p $OUT; : > $OUT/summary.txt
for pass in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-steps 0 $v > $OUT/v${i}_p$pass.log 2>&1 || exit 1
    grep '^{' $OUT/v${i}_p$pass.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pass $pass [$v]', d['value'], d['ms_per_step'])" >> $OUT/summary.txt
  done
done
