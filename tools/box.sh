#!/bin/bash
# GPU box (through gpurun): every measurement step of a round in one parameterised script.  Each
# step runs under its own time limit; the script stops at the first failing step and records
# every step's exit code in gpurun_out/<TAG>/status.txt.
# usage: tools/box.sh TAG step...
#   pytest[=files]     the -m gpu suite (or the named test files)
#   smoke              __graft_entry__.smoke()
#   c2 c3 c3sp c3spd ent c5 off dense gw1 e2e train
#                      bench lines: C2 (with the CPU baseline and the e2e leg), C3 (host pre-split),
#                      C3 GPT-2 + specials found on the host / on the device, the low-repetition
#                      corpus, C5 stress, both memo shortcuts off, a special-dense corpus, the
#                      world-1 gather step, the PCIe-inclusive leg alone, the trainer
#   prof_<cfg>         rocprofv3 kernel trace + one PMC pass per counter group (tools/profile_gpu.sh)
#   ab=spec,spec,...   kernel-trace A/B of library variants / bench args (tools/gpu_ab_trace.sh)
#   stamps=lib[:kind]  per-phase cycle stamps of an SW_STAMPS build (tools/phase_stamps.py)
#   pmc=lib[@args]     one PMC pass of instruction counters over the C2 bench (or its args) with library `lib`
set -u
TAG=$1; shift
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
bench() {  # name args...
  local name=$1; shift
  run "bench_$name" 400 python -u bench.py "$@"
}
NB=(--no-cpu-baseline --e2e-steps 0 --small-steps 0)
for s in "$@"; do
  case $s in
    pytest) run pytest 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    pytest=*) v=${s#pytest=}; run pytest_part 900 python -u -m pytest ${v//+/ } -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    c2) bench c2 --steps 20 --warmup 2 ;;
    c3) bench c3 --steps 20 --warmup 2 --presplit host "${NB[@]}" ;;
    c3sp) bench c3sp --steps 20 --warmup 2 --presplit host --pattern gpt2 --specials 1 ;;
    c3spd) bench c3spd --steps 20 --warmup 2 --pattern gpt2 --specials 1 --specials-device ;;
    ent) bench ent --steps 20 --warmup 2 --corpus entropy "${NB[@]}" ;;
    c5) bench c5 --steps 20 --warmup 2 --config c5 "${NB[@]}" ;;
    off) bench off --steps 10 --warmup 2 --no-dedupe --no-chunk-table "${NB[@]}" ;;
    dense) bench dense --steps 10 --warmup 2 --pattern gpt2 --specials 64 --specials-device "${NB[@]}" ;;
    gw1) bench gw1 --steps 10 --warmup 2 --gather-world1 "${NB[@]}" ;;
    e2e) bench e2e --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 3 ;;
    train) run bench_train 400 python -u tools/bench_train.py --workloads toy500,mixed32m,mixed128m --no-cpu ;;
    prof_c2) run prof_c2 1100 bash tools/profile_gpu.sh "${TAG}_c2" ;;
    prof_c3) run prof_c3 1100 bash tools/profile_gpu.sh "${TAG}_c3" --presplit host ;;
    prof_c5) run prof_c5 1100 bash tools/profile_gpu.sh "${TAG}_c5" --config c5 ;;
    prof_c3sp) run prof_c3sp 1100 bash tools/profile_gpu.sh "${TAG}_c3sp" --presplit host --pattern gpt2 --specials 1 ;;
    prof_c3spd) run prof_c3spd 1100 bash tools/profile_gpu.sh "${TAG}_c3spd" --pattern gpt2 --specials 1 --specials-device ;;
    prof_ent) run prof_ent 1100 bash tools/profile_gpu.sh "${TAG}_ent" --corpus entropy ;;
    prof_off) run prof_off 1100 bash tools/profile_gpu.sh "${TAG}_off" --no-dedupe --no-chunk-table ;;
    prof_dense) run prof_dense 1100 bash tools/profile_gpu.sh "${TAG}_dense" --pattern gpt2 --specials 64 --specials-device ;;
    ab=*) IFS=',' read -r -a specs <<< "${s#ab=}"
          specs=("${specs[@]//+/,}")  # (a spec's own bench args: lib.so@--corpus+entropy)
          run "ab" 1000 bash tools/gpu_ab_trace.sh "$TAG" "${specs[@]}" ;;
    stamps=*) v=${s#stamps=}; lib=${v%%:*}; kind=mixed; [ "$lib" != "$v" ] && kind=${v#*:}
              run "stamps_${lib%.so}_$kind" 200 env SHREDWORD_HIP_LIB="$R/shredword_amd/$lib" \
                python3 tools/phase_stamps.py 250000 "$kind" fused ;;
    pmc=*) v=${s#pmc=}; lib=${v%%@*}; extra=""; [ "$lib" != "$v" ] && extra=${v#*@} && extra=${extra//+/ }
           nm=pmc_$(echo "${v%.so}" | tr -c 'A-Za-z0-9_\n' '_')
           (cd /tmp && export TMPDIR=/tmp && SHREDWORD_HIP_LIB="$R/shredword_amd/$lib" timeout -k 10 300 rocprofv3 --pmc \
              SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
              -d "$O/$nm" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 "${NB[@]}" $extra \
              > "$O/$nm.log" 2>&1)
           rc=$?; echo "$nm rc=$rc" >> "$O/status.txt"; [ $rc -eq 0 ] || exit $rc ;;
    fetch=*) v=${s#fetch=}; lib=${v%%@*}; extra=""; [ "$lib" != "$v" ] && extra=${v#*@} && extra=${extra//+/ }
             nm=$(echo "${v}" | tr -c 'A-Za-z0-9_\n' '_')
             for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
               g=$(echo $grp | cut -d' ' -f1)
               (cd /tmp && export TMPDIR=/tmp && SHREDWORD_HIP_LIB="$R/shredword_amd/$lib" timeout -k 10 300 rocprofv3 --pmc $grp \
                  -d "$O/fetch_${nm}_$g" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 "${NB[@]}" $extra \
                  > "$O/fetch_${nm}_$g.log" 2>&1)
               rc=$?; echo "fetch_${nm}_$g rc=$rc" >> "$O/status.txt"; [ $rc -eq 0 ] || exit $rc
             done ;;
    diag=*) v=${s#diag=}; extra=""; [ "$v" != "" ] && extra=${v//+/ }  # (latency / TLB / TA diagnostics of a bench config)
            i=0
            for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" \
                       "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" \
                       "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
              i=$((i+1))
              (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $grp -d "$O/diag$i" -o run --output-format csv \
                 -- python3 "$R/bench.py" --steps 2 --warmup 1 "${NB[@]}" $extra > "$O/diag$i.log" 2>&1)
              rc=$?; echo "diag$i rc=$rc" >> "$O/status.txt"; [ $rc -eq 0 ] || exit $rc
            done ;;
    *) echo "unknown step $s" >> "$O/status.txt"; exit 2 ;;
  esac
done
echo all-done >> "$O/status.txt"
