#!/usr/bin/env python3
"""Summary of a tools/gpu_ab_trace.sh run: value, kernel_ms and the chosen kernels' average times.
usage: tools/ab_summary.py gpurun_out/abt_TAG [kernel substrings...]"""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
keys = sys.argv[2:] or ["split_classify", "k_edges", "k_classify", "k_presplit_bits", "k_compact"]
for log in sorted(glob.glob(os.path.join(out, "*.log"))):
    name = os.path.basename(log)[:-4]
    f = glob.glob("%s/%s/**/run_kernel_stats.csv" % (out, name), recursive=True)
    if not f:
        continue
    rows = list(csv.DictReader(open(f[0])))
    line = [l for l in open(log) if l.startswith("{")]
    d = json.loads(line[-1]) if line else {}
    ks = [r for r in rows if any(k in r["Name"] for k in keys)]
    print("== %-28s value %-10s kernel_ms %-7s | %s" % (
        name, d.get("value"), d.get("roofline", {}).get("kernel_ms"),
        " ".join("%s=%.4f" % (r["Name"].split("(")[0].replace("sw::", "")[:22], float(r["AverageNs"]) / 1e6)
                 for r in ks)))
