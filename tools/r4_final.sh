#!/bin/bash
# GPU box, round 4: the bench lines (C2 headline with CPU baseline + e2e, C3 GPT-2 + specials on
# the host, C3 plain, the low-repetition corpus, C5 stress, memo shortcuts off) and the trainer,
# then (step "prof") the rocprofv3 trace + PMC passes of each.  Every step has its own limit; the
# script stops at the first failing step.
# usage: tools/r4_final.sh TAG [steps...]  steps: smoke c2 c3sp c3 ent c5 off train prof_* (default: benches)
set -u
TAG=${1:-r4}; shift || true
STEPS=${*:-"smoke c2 c3sp c3 ent c5 off train"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  (cd "$R" && timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1)
  local rc=$?
  echo "$name rc=$rc" >> "$O/status.txt"
  [ $rc -eq 0 ] || exit $rc
}
prof() {  # tag bench args...
  local t=$1; shift
  timeout -k 10 1100 bash "$R/tools/profile_gpu.sh" "${TAG}_$t" "$@" > "$O/prof_$t.log" 2>&1
  local rc=$?
  echo "prof_$t rc=$rc" >> "$O/status.txt"
  [ $rc -eq 0 ] || exit $rc
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    c2) run bench_c2 400 python -u bench.py --steps 20 --warmup 2 ;;
    c3sp) run bench_c3sp 400 python -u bench.py --steps 20 --warmup 2 --presplit host --pattern gpt2 --specials 1 ;;
    c3) run bench_c3 400 python -u bench.py --steps 20 --warmup 2 --presplit host --no-cpu-baseline --e2e-steps 0 ;;
    ent) run bench_ent 400 python -u bench.py --steps 20 --warmup 2 --corpus entropy --no-cpu-baseline --e2e-steps 0 ;;
    c5) run bench_c5 400 python -u bench.py --steps 20 --warmup 2 --config c5 --no-cpu-baseline --e2e-steps 0 ;;
    off) run bench_off 400 python -u bench.py --steps 10 --warmup 2 --no-dedupe --no-chunk-table --no-cpu-baseline --e2e-steps 0 ;;
    train) run bench_train 400 python -u tools/bench_train.py --workloads toy500,mixed32m,mixed128m --no-cpu ;;
    prof_c2) prof c2 ;;
    prof_c5) prof c5 --config c5 ;;
    prof_c3sp) prof c3sp --presplit host --pattern gpt2 --specials 1 ;;
    prof_ent) prof ent --corpus entropy ;;
    prof_off) prof off --no-dedupe --no-chunk-table ;;
    prof_train)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/train_trace" -o run \
         --output-format csv -- python3 "$R/tools/bench_train.py" --workloads mixed128m --no-cpu > "$O/train_trace.log" 2>&1)
      rc=$?; echo "train_trace rc=$rc" >> "$O/status.txt"; [ $rc -eq 0 ] || exit $rc
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $grp -d "$O/train_pmc$i" -o run \
           --output-format csv -- python3 "$R/tools/bench_train.py" --workloads mixed128m --no-cpu > "$O/train_pmc$i.log" 2>&1)
        rc=$?; echo "train_pmc$i rc=$rc" >> "$O/status.txt"; [ $rc -eq 0 ] || exit $rc
      done ;;
    *) echo "unknown step $s" >> "$O/status.txt"; exit 2 ;;
  esac
done
echo all-done >> "$O/status.txt"
