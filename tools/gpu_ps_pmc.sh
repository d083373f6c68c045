#!/bin/bash
# GPU box: SQ counters of k_presplit (tools/ps_time.py) for the default library and each
# variant given.  Summary: gpurun_out/ps_pmc/summary.txt
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ps_pmc; mkdir -p "$OUT"
export TMPDIR=/tmp
CNT="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD"
for lib in default "$@"; do
  if [ "$lib" = default ]; then unset SHREDWORD_HIP_LIB; else export SHREDWORD_HIP_LIB=$R/shredword_amd/$lib; fi
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT -d "$OUT/$lib" -o run --output-format csv -- python3 "$R/tools/ps_time.py" > "$OUT/$lib.log" 2>&1
  rc=$?; echo "$lib rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY' > "$OUT/summary.txt"
import collections, csv, glob, os, sys
out = sys.argv[1]
for d in sorted(glob.glob(out + "/*/")):
    f = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not f: continue
    per = collections.defaultdict(float); disp = set()
    for r in csv.DictReader(open(f[0])):
        if "k_presplit" not in r["Kernel_Name"]: continue
        per[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    n = max(1, len(disp))
    print(os.path.basename(d.rstrip("/")), "dispatches", n)
    for k in sorted(per): print("   %-22s %.4g" % (k, per[k] / n))
PY
cat "$OUT/summary.txt"
