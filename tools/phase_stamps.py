#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of the encode kernels from the SW_STAMPS build (GPU box).
usage: SHREDWORD_HIP_LIB=shredword_amd/libshredword_hip_stamps.so python tools/phase_stamps.py [n_strings]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from shredword_amd import Tokenizer, _lib, corpus  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 250_000
kind = corpus.STRESS if (len(sys.argv) > 2 and sys.argv[2] == "stress") else corpus.MIXED
model = "bl50k.model" if kind == corpus.STRESS else "bl32k.model"
buf, off = corpus.synth(1_000_003, kind, n, 1074 if kind == corpus.MIXED else 600, n_threads=16)
bits, nch = corpus.presplit(buf, off, 0, n_threads=16)
if len(sys.argv) > 3 and sys.argv[3] == "fused":  # the device pre-split inside k_split_classify
    bits = None
tok = Tokenizer(0)
tok.load(os.path.join(ROOT, "tests", "golden", model))
tok.encode_packed(buf, off, bits)  # warm
L = _lib.lib()
out = (ctypes.c_double * 32)()
_lib.check(L.sw_encoder_phase_cycles(tok._encoder(), out, 1))
reps = 3
for _ in range(reps):
    tok.encode_packed(buf, off, bits)
_lib.check(L.sw_encoder_phase_cycles(tok._encoder(), out, 1))
tiles = (len(buf) + 2047) // 2048
names = {0: "classify: stage+enum", 1: "classify: lookups", 7: "classify: dedupe", 2: "classify: counts",
         3: "classify: strings",
         4: "merge N<16 (blk)", 5: "merge N>=16 (blk)", 6: "merge long (blk)",
         12: "fused: stage+strings", 13: "fused: class masks", 14: "fused: rules",
         8: "compact: prologue loads", 9: "compact: slots+gathers", 10: "compact: scan+stores", 11: "compact: strings"}
tot = sum(out[i] for i in names)
print("kind=%s bytes=%d chunks=%d tiles=%d kernel_ms=%.3f" % (model, len(buf), nch, tiles, tok.last_stats.ms_kernels))
for i, nm in names.items():
    print("%-26s %12.0f cycles/tile-equiv  %5.1f%%" % (nm, out[i] / tiles / reps, 100 * out[i] / tot))
