#!/usr/bin/env python3
"""Trainer benchmark: the GPU trainer (shredword_amd.BPETrainer) against
its CPU oracle (oracle/sw_train_oracle.c, 1 thread; the reference trainer's algorithm restated)
and, when oracle/_ref/libtrainer.so was built (`make -C oracle ref`, container), the reference
trainer itself (a child process; its per-merge printf output discarded), on seeded synthetic
corpora.  One JSON line per workload:
  {"workload", "corpus_bytes", "words", "symbols", "merges", "gpu_s", "gpu_breakdown_ms",
   "cpu_s", "speedup", "same_merges", "reference_s", "speedup_vs_reference"}
Times cover corpus load + training (+ the reference's file read).
usage: python tools/bench_train.py [--workloads toy500,mixed32m] [--no-cpu] [--reference-on toy500]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import shredword_amd as sa  # noqa: E402
from shredword_amd import corpus  # noqa: E402

WORKLOADS = {
    # the toy500 recipe (oracle/make_golden.py): 10 MB ASCII, 500 merges, min_pair_freq 2
    "toy500": ({"seed": 1001, "kind": corpus.ASCII, "strings": 10000, "mean": 1000}, (756, 0, 0.9999, 2)),
    # 32 MB of mixed UTF-8, 4000 merges
    "mixed32m": ({"seed": 77, "kind": corpus.MIXED, "strings": 30000, "mean": 1074}, (4256, 0, 0.995, 2)),
    # 128 MB of mixed UTF-8, 8000 merges (GPU only unless --cpu-big)
    "mixed128m": ({"seed": 78, "kind": corpus.MIXED, "strings": 120000, "mean": 1074}, (8256, 0, 0.995, 2)),
}


def text_of(rec):
    buf, _ = corpus.synth(rec["seed"], rec["kind"], rec["strings"], rec["mean"], n_threads=16)
    return bytes(buf).replace(b"\0", b" ")


REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libtrainer.so")
REF_CHILD = """
import ctypes, sys, time
L = ctypes.CDLL(sys.argv[1])
class Cfg(ctypes.Structure):
    _fields_ = [("target_vocab_size", ctypes.c_size_t), ("unk_id", ctypes.c_int32),
                ("character_coverage", ctypes.c_float), ("min_pair_freq", ctypes.c_uint64)]
L.create_trainer.restype = ctypes.c_void_p
L.create_trainer.argtypes = [ctypes.POINTER(Cfg)]
L.bpe_load_corpus.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
L.bpe_train.argtypes = [ctypes.c_void_p]
c = Cfg(int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5]), int(sys.argv[6]))
t0 = time.perf_counter()
t = L.create_trainer(ctypes.byref(c))
assert L.bpe_load_corpus(t, sys.argv[2].encode()) == 0
n = L.bpe_train(t)
sys.stderr.write("REF %d %.6f\\n" % (n, time.perf_counter() - t0))
"""


def time_reference(text, cfg):
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "corpus.txt")
        with open(path, "wb") as f:
            f.write(text)
        r = subprocess.run([sys.executable, "-c", REF_CHILD, REF_LIB, path] + [str(x) for x in cfg],
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=3000)
        for ln in r.stderr.decode(errors="replace").splitlines():
            if ln.startswith("REF "):
                _, n, s = ln.split()
                return int(n), float(s)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="toy500,mixed32m")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-big", action="store_true", help="also time the CPU baselines on mixed128m")
    ap.add_argument("--reference-on", default="toy500", help="workloads the reference trainer is timed on")
    args = ap.parse_args()
    for name in args.workloads.split(","):
        rec, cfg = WORKLOADS[name]
        text = text_of(rec)
        t = sa.BPETrainer(*cfg)
        t0 = time.perf_counter()
        t.load_text(text)
        n = t.train()
        gpu_s = time.perf_counter() - t0
        st = t.stats
        rows = t.merges
        line = {"workload": name, "corpus_bytes": len(text), "config": list(cfg), "words": int(st["words"]),
                "symbols": int(st["symbols"]), "merges": n, "gpu_s": round(gpu_s, 4),
                "gpu_breakdown_ms": {k: round(v, 2) for k, v in st.items() if k.startswith("ms_")},
                "ms_per_merge_device": round(st["ms_rewrites"] / max(n, 1), 4),
                "merges_sha1": hashlib.sha1(np.ascontiguousarray(rows, dtype=np.int64).tobytes()).hexdigest(),
                "launch_ahead": os.environ.get("SW_TRAIN_NO_AHEAD", "0") != "1"}
        if not args.no_cpu and (name != "mixed128m" or args.cpu_big):
            import oracle
            c0 = time.perf_counter()
            exp, _ = oracle.train(text, *cfg)
            cpu_s = time.perf_counter() - c0
            line.update({"cpu_s": round(cpu_s, 3), "cpu_kind": "port (oracle/sw_train_oracle.c, 1 thread)",
                         "speedup": round(cpu_s / gpu_s, 2), "same_merges": bool(np.array_equal(exp, rows))})
        print("# %s: gpu %.3f s, timing the CPU baselines" % (name, gpu_s), file=sys.stderr, flush=True)
        if name in args.reference_on.split(",") and os.path.exists(REF_LIB):
            rn, rs = time_reference(text, cfg)
            if rs is not None:
                line.update({"reference_s": round(rs, 3), "reference_merges": rn,
                             "speedup_vs_reference": round(rs / gpu_s, 2)})
        print(json.dumps(line), flush=True)
        t.destroy()


if __name__ == "__main__":
    main()
