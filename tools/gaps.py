"""Per-launch timeline of the encode pipeline from a rocprofv3 kernel trace: each kernel's
duration and the idle gap before it, for the last full launch (k_tile_strings .. k_string_offsets).
usage: python tools/gaps.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_tile_strings" in r["Kernel_Name"]]
ends = [i for i, r in enumerate(rows) if "k_string_offsets" in r["Kernel_Name"]]
for s in starts[-2:]:
    e = min(i for i in ends if i > s)
    pre = s - 1 if s > 0 and "k_presplit_bits" in rows[s - 1]["Kernel_Name"] else s
    seq = rows[pre:e + 1]
    t0 = int(seq[0]["Start_Timestamp"])
    prev_end = t0
    busy = gap = 0
    for r in seq:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        g = max(0, a - prev_end)
        gap += g
        busy += b - a
        print("%-50s %8.1f us  gap %6.1f us" % (r["Kernel_Name"][:50], (b - a) / 1e3, g / 1e3))
        prev_end = max(prev_end, b)
    print("launch: span %.1f us, kernels %.1f us, gaps %.1f us\n" % ((prev_end - t0) / 1e3, busy / 1e3, gap / 1e3))
