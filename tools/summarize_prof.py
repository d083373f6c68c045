#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh output directory into profiles/<tag>.md (+ the rocprofv3
kernel-stats CSV and a JSON of the counters).

The encode pipeline is one sw_encode_device call = several kernels; per-launch figures are the
per-dispatch means times the dispatches per launch (launches = k_classify dispatches).  HBM
traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KB; FETCH_SIZE
under-reports wide coalesced streaming reads by 2x on gfx950, so both the raw and the
x2-corrected read figure are shown (the corrected one is an upper bound here, since much of
this pipeline's traffic is not 16-B-per-lane streaming reads)."""
import collections
import csv
import glob
import json
import os
import shutil
import sys


TRAFFIC_KEY = ("n_bytes", "merges", "pattern", "chunk_table", "dedupe", "presplit", "corpus", "specials",
               "specials_found")


def pmc(dirpath):
    """{kernel: {counter: mean per dispatch}}, {kernel: dispatches}"""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(dirpath, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].replace("void ", "")
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(out, tag + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats_csv)))
    calls = {r["Name"].split("(")[0].replace("void ", ""): int(r["Calls"]) for r in rows}
    # one classification dispatch per launch: k_classify (host bitmap) or k_split_classify (fused)
    launches = max([1] + [v for k, v in calls.items() if k.split("<")[0] in ("sw::k_classify", "sw::k_split_classify")])

    # kernel families whose member is chosen per launch (the compaction: k_compact, k_compact7<.., typed>,
    # the first launch without the last launch's statistics takes k_compact): the member with the
    # most dispatches stands for the family, counted once per launch
    def family(name):
        return "sw::k_compact" if name.startswith(("sw::k_compact<", "sw::k_compact7<")) else name
    fam_calls, fam_rep = collections.Counter(), {}
    for k, v in calls.items():
        fam_calls[family(k)] += v
        if family(k) not in fam_rep or v > calls[fam_rep[family(k)]]:
            fam_rep[family(k)] = k

    def per_launch(name):  # dispatches of a kernel per encode launch (bench.py's one extra
        # k_presplit + k_popcount outside the timed steps, for the chunk count, is not one)
        f = family(name)
        if f != name:
            return max(1, int(round(fam_calls[f] / launches))) if fam_rep.get(f) == name and fam_calls[f] >= launches else 0
        return max(1, int(round(calls.get(name, launches) / launches))) if calls.get(name, 0) >= launches else 0

    per_launch_ms = sum(float(r["AverageNs"]) * per_launch(r["Name"].split("(")[0].replace("void ", ""))
                        for r in rows if r["Name"].startswith(("sw::", "void sw::"))) / 1e6
    spans = []  # wall span of each launch (k_tile_strings start .. k_string_offsets end): the
    # merge kernels run side by side on forked streams, so the kernel-time sum over-counts them
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                     for r in csv.DictReader(open(tr))), key=lambda x: x[0])
        t_start = None
        for a0, b0, nm in ev:
            if "k_tile_strings" in nm:
                t_start = a0
            elif "k_string_offsets" in nm and t_start is not None:
                spans.append((b0 - t_start) / 1e6)
                t_start = None
    span_txt = ("  Wall span per launch (first kernel start to last kernel end, from the kernel trace): "
                "**%.3f ms** median, %.3f ms min over %d launches (the first includes one-time setup)." % (
                    sorted(spans)[len(spans) // 2], min(spans), len(spans))
                if spans else "")
    lines = ["# rocprofv3 summary: %s" % tag, "",
             "Command: `tools/profile_gpu.sh %s` (bench.py --steps 3 --warmup 1 --no-cpu-baseline; kernel trace + "
             "stats pass, then one rocprofv3 --pmc pass per counter group)." % tag, "",
             "Encode launches traced: %d.  Sum of the pipeline's kernel time per launch: **%.3f ms** "
             "(per launch = average x dispatches per launch; bench.py's one extra pre-split for the "
             "chunk count, outside the timed steps, is not counted)." % (launches, per_launch_ms) + span_txt, "",
             "| kernel | calls | avg ms | per launch ms | % |", "|---|---|---|---|---|"]
    for r in rows:
        nm = r["Name"].split("(")[0].replace("void ", "")
        lines.append("| %s | %s | %.4f | %.4f | %.2f |" % (
            r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1e6,
            float(r["AverageNs"]) * per_launch(nm) / 1e6, float(r["Percentage"])))
    c = pmc(src)
    tot = collections.defaultdict(float)
    if c:
        cnames = sorted({n for k in c.values() for n in k})
        lines += ["", "PMC, mean per dispatch:", "", "| kernel | " + " | ".join(cnames) + " |",
                  "|---|" + "---|" * len(cnames)]
        for k in sorted(c):
            if not k.startswith("sw::"):
                continue
            lines.append("| %s | " % k[:48] + " | ".join("%.4g" % c[k].get(n, float("nan")) for n in cnames) + " |")
            per = per_launch(k)
            for n in cnames:
                tot[n] += c[k].get(n, 0.0) * per
    derived = {"pipeline_ms_per_launch": per_launch_ms}
    if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
        derived["hbm_read_bytes_raw"] = tot["FETCH_SIZE"] * 1024
        derived["hbm_read_bytes_x2"] = tot["FETCH_SIZE"] * 2048
        derived["hbm_write_bytes"] = tot["WRITE_SIZE"] * 1024
        derived["traffic_bytes_per_launch"] = derived["hbm_read_bytes_raw"] + derived["hbm_write_bytes"]
        derived["traffic_bytes_per_launch_x2"] = derived["hbm_read_bytes_x2"] + derived["hbm_write_bytes"]
    if tot.get("TCC_HIT_sum"):
        derived["l2_hit_rate"] = tot["TCC_HIT_sum"] / max(1.0, tot["TCC_HIT_sum"] + tot.get("TCC_MISS_sum", 0))
    lines += ["", "Pipeline totals per launch (sum over kernels x dispatches per launch):", "", "```",
              json.dumps({k: v for k, v in tot.items()}, indent=1), json.dumps(derived, indent=1), "```"]
    with open(os.path.join(out, tag + ".md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out, tag + "_pmc.json"), "w") as f:
        json.dump({"per_kernel": c, "per_launch": tot, "derived": derived}, f, indent=1)
    # bench.py quotes roofline.traffic from profiles/traffic.json when its workload matches
    bench = None
    for ln in open(os.path.join(src, "trace.log"), errors="replace"):
        if ln.startswith("{") and '"metric"' in ln:
            bench = json.loads(ln)
    if bench and "traffic_bytes_per_launch" in derived:  # one entry per workload, keyed as bench.py matches it
        cfg = bench["config"]
        entry = {"source": "profiles/%s.md" % tag, "n_bytes": cfg["bytes_per_rank"], "merges": cfg["merges"],
                 "pattern": cfg["pattern"], "chunk_table": cfg.get("chunk_table"), "dedupe": cfg.get("dedupe"),
                 "presplit": cfg.get("presplit", "host"), "corpus": cfg.get("corpus", "mixed"),
                 "specials": (bench.get("specials") or {}).get("per_kib", 0.0),
                 "specials_found": (bench.get("specials") or {}).get("found", "host"),
                 "traffic_bytes_per_launch": derived["traffic_bytes_per_launch"],
                 "traffic_bytes_per_launch_x2": derived["traffic_bytes_per_launch_x2"],
                 # the LDS bank-conflict and VALU counters beside the bytes
                 "counters": {"valu_wave_insts": tot.get("SQ_INSTS_VALU"),
                              "valu_issue_floor_ms": (tot["SQ_INSTS_VALU"] * 2 / 1024 / 2.4e6
                                                      if "SQ_INSTS_VALU" in tot else None),
                              "lds_insts": tot.get("SQ_INSTS_LDS"),
                              "lds_bank_conflict_cycles": tot.get("SQ_LDS_BANK_CONFLICT"),
                              "lds_conflict_cycles_per_lds_inst": (
                                  tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_INSTS_LDS"] if tot.get("SQ_INSTS_LDS") else None),
                              "wait_fraction_of_wave_cycles": (
                                  tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"] if tot.get("SQ_WAVE_CYCLES") else None),
                              "l2_hit_rate": derived.get("l2_hit_rate"),
                              "note": "pipeline totals per launch; VALU floor = wave instructions x 2 cycles / "
                                      "1024 SIMDs / 2.4 GHz"}}
        # the dominant kernel alone (bench.py roofline.dominant): its trace time and its own bytes
        cls = [k for k in c if k.split("<")[0] in ("sw::k_split_classify", "sw::k_classify")]
        if cls:
            k = max(cls, key=lambda n: calls.get(n, 0))
            avg = [float(r["AverageNs"]) / 1e6 for r in rows if r["Name"].split("(")[0].replace("void ", "") == k]
            fb, wb = c[k].get("FETCH_SIZE"), c[k].get("WRITE_SIZE")
            entry["dominant"] = {
                "kernel": k, "avg_ms": round(avg[0], 4) if avg else None,
                "fetch_bytes": fb * 1024 if fb is not None else None, "write_bytes": wb * 1024 if wb is not None else None,
                "traffic_bytes": (fb + wb) * 1024 if fb is not None and wb is not None else None,
                "lds_conflict_cycles_per_lds_inst": (c[k]["SQ_LDS_BANK_CONFLICT"] / c[k]["SQ_INSTS_LDS"]
                                                     if c[k].get("SQ_INSTS_LDS") else None),
                "valu_wave_insts": c[k].get("SQ_INSTS_VALU"),
                "wait_fraction_of_wave_cycles": (c[k]["SQ_WAIT_ANY"] / c[k]["SQ_WAVE_CYCLES"]
                                                 if c[k].get("SQ_WAVE_CYCLES") else None)}
        path = os.path.join(out, "traffic.json")
        try:
            tj = json.load(open(path))
        except (OSError, ValueError):
            tj = {}
        entries = tj.get("entries", [])
        key = lambda e: tuple(e.get(k) for k in TRAFFIC_KEY)  # noqa: E731
        entries = [e for e in entries if key(e) != key(entry)] + [entry]
        with open(path, "w") as f:
            json.dump({"note": "per workload: FETCH_SIZE+WRITE_SIZE summed over the pipeline's kernels per launch "
                               "(raw FETCH; _x2 doubles FETCH per the gfx950 wide-read correction); bench.py quotes "
                               "the entry whose key fields match its workload", "key": list(TRAFFIC_KEY),
                       "entries": entries}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
