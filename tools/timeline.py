"""Print one launch's kernel timeline from a rocprofv3 kernel-trace CSV.
usage: python tools/timeline.py DIR [anchor_kernel_substring] [which (negative: from the end)]"""
import csv
import glob
import sys

d = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_tile_strings"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
f = glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = idx[which]
i1 = idx[which + 1] if which + 1 < 0 or which + 1 < len(idx) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%9.3f %9.3f %8.3f s=%s %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, r["Stream_Id"], r["Kernel_Name"][:70]))
