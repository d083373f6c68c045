#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh output directory into profiles/<tag>.md (+ copies of the
rocprofv3 kernel-stats CSV).  HBM traffic per launch follows MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are KB; FETCH_SIZE under-reports wide coalesced streaming reads by 2x on
gfx950, so both the raw and the x2-corrected read figure are shown (the corrected one is an upper
bound for this kernel, whose reads are not all wide streaming reads)."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

KERNEL = "k_encode_tiles"


def pmc(dirpath):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(dirpath, "pmc*", "run_counter_collection.csv"))):
        per_dispatch = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                per_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d in per_dispatch.values():
            for c, v in d.items():
                vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(out, tag + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats_csv)))
    c = pmc(src)
    lines = ["# rocprofv3 summary: %s" % tag, "", "Command: `tools/profile_gpu.sh %s` (bench.py --steps 3 --warmup 1, "
             "kernel trace + stats pass, then one pass per counter group)." % tag, "",
             "| kernel | calls | avg ms | % |", "|---|---|---|---|"]
    for r in rows:
        lines.append("| %s | %s | %.4f | %.2f |" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                   float(r["Percentage"])))
    lines += ["", "PMC, %s, mean per dispatch:" % KERNEL, "", "| counter | value |", "|---|---|"]
    for k in sorted(c):
        lines.append("| %s | %.4g |" % (k, c[k]))
    derived = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        derived["hbm_read_bytes_raw"] = c["FETCH_SIZE"] * 1024
        derived["hbm_read_bytes_x2"] = c["FETCH_SIZE"] * 2048
        derived["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        derived["traffic_bytes_per_launch"] = derived["hbm_read_bytes_raw"] + derived["hbm_write_bytes"]
    if "TCC_HIT_sum" in c:
        derived["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0))
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        derived["wave_wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    kavg = [float(r["AverageNs"]) for r in rows if KERNEL in r["Name"]]
    if "GRBM_GUI_ACTIVE" in c and kavg:
        derived["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / kavg[0]
    lines += ["", "Derived:", "", "```", json.dumps(derived, indent=1), "```"]
    with open(os.path.join(out, tag + ".md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out, tag + "_pmc.json"), "w") as f:
        json.dump({"kernel": KERNEL, "counters": c, "derived": derived}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
