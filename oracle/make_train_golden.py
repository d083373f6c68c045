#!/usr/bin/env python3
"""Generate the trainer fixtures under tests/golden/ (train_*.bin, train_*.freq.npy,
train_index.json) by running the REFERENCE's own C++ trainer.

CONTAINER-ONLY test infrastructure.  Needs oracle/_ref/libtrainer.so, built from the reference
sources in place by `make -C oracle ref`, and shredword_amd/libshredword_hip.so for the seeded
synthetic corpora.  Only the outputs (merge rows, token frequencies, recipes) are committed.

The reference leaves Symbol.deleted uninitialised (histogram.cpp:14-22), so its result depends
on what the allocator hands it: recycled chunks with a non-zero byte there make symbols start
"deleted" (tests/golden/toy500.bin, made without this, diverges from a clean run at merge 151).
Each run here therefore sets glibc's MALLOC_PERTURB_=255 with the per-thread cache off
(GLIBC_TUNABLES=glibc.malloc.tcache_count=0: its fast path skips the perturbation), which makes
every allocation start zeroed: the run then computes the trainer's intended behaviour, the one oracle/sw_train_oracle.c
restates with that defect fixed.  The vocabulary file's frequencies are parsed knowing each
token's C string (tokens may hold '\\n').  unk_id stays >= 0 (bpe.cpp:709 writes freq[-1]
otherwise); NUL bytes in a synthetic corpus become spaces.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

from shredword_amd import corpus  # noqa: E402  (synthetic inputs only)

# name, corpus recipe, BPEConfig(target_vocab_size, unk_id, character_coverage, min_pair_freq)
RECIPES = [
    ("toy500", {"seed": 1001, "kind": "ascii", "strings": 10000, "mean": 1000}, (756, 0, 0.9999, 2)),
    ("mixed1k", {"seed": 7, "kind": "mixed", "strings": 3000, "mean": 500}, (1256, 0, 0.995, 2)),
    ("minfreq", {"seed": 5, "kind": "ascii", "strings": 3000, "mean": 400}, (4256, 0, 0.9999, 40)),
    ("runs", {"file": "train_runs.txt"}, (456, 0, 0.9999, 2)),
    ("unk7", {"seed": 11, "kind": "stress", "strings": 400, "mean": 600}, (856, 7, 0.98, 3)),
]
KINDS = {"ascii": corpus.ASCII, "mixed": corpus.MIXED, "stress": corpus.STRESS}


def runs_text():
    """Repeated symbols and alternations: (a,a) runs, overlapping candidates, long words."""
    rng = np.random.default_rng(3)
    words = []
    for _ in range(4000):
        k = int(rng.integers(0, 6))
        n = int(rng.integers(1, 24))
        if k == 0:
            words.append("a" * n)
        elif k == 1:
            words.append("ab" * n)
        elif k == 2:
            words.append("aab" * (n // 2 + 1))
        elif k == 3:
            words.append("".join("xyz"[int(c)] for c in rng.integers(0, 3, size=n)))
        elif k == 4:
            words.append("ba" * n + "a")
        else:
            words.append("q" + "a" * n + "q")
    seps = [" ", "\n", "\t", "  ", "\r\n"]
    return "".join(w + seps[int(rng.integers(0, len(seps)))] for w in words).encode()


def corpus_bytes(rec):
    if "file" in rec:
        return open(os.path.join(GOLD, rec["file"]), "rb").read()
    buf, _ = corpus.synth(rec["seed"], KINDS[rec["kind"]], rec["strings"], rec["mean"])
    return bytes(buf).replace(b"\0", b" ")  # (the reference's line reader stops at NUL bytes)


def token_cstrings(rows):
    """bpe_save's token strings (bpe.cpp:686-701): C strings, so byte 0 is "" and a merge
    concatenates its members up to their first NUL."""
    toks = [bytes([i]) if i else b"" for i in range(256)]
    for a, b, _ in rows:
        toks.append(toks[a] + toks[b])
    return toks


def parse_vocab(raw, toks):
    freq, pos = [], 0
    for t in toks:
        assert raw[pos:pos + len(t)] == t, (len(freq), raw[pos:pos + 40])
        pos += len(t) + 1
        end = raw.index(b"\n", pos)
        freq.append(int(raw[pos:end]))
        pos = end + 1
    assert pos == len(raw)
    return np.array(freq, dtype=np.uint64)


def run_reference(text, cfg):
    lib = os.path.join(ROOT, "oracle", "_ref", "libtrainer.so")
    with tempfile.TemporaryDirectory() as td:
        cpath, mpath, vpath = (os.path.join(td, f) for f in ("corpus.txt", "m.bin", "v.txt"))
        with open(cpath, "wb") as f:
            f.write(text)
        code = f"""
import ctypes
L = ctypes.CDLL({lib!r})
class Cfg(ctypes.Structure):
    _fields_ = [("target_vocab_size", ctypes.c_size_t), ("unk_id", ctypes.c_int32),
                ("character_coverage", ctypes.c_float), ("min_pair_freq", ctypes.c_uint64)]
L.create_trainer.restype = ctypes.c_void_p
L.create_trainer.argtypes = [ctypes.POINTER(Cfg)]
L.bpe_load_corpus.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
L.bpe_train.argtypes = [ctypes.c_void_p]
L.bpe_save.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
c = Cfg(*{tuple(cfg)!r})
t = L.create_trainer(ctypes.byref(c))
assert L.bpe_load_corpus(t, {cpath!r}.encode()) == 0
assert L.bpe_train(t) >= 0
L.bpe_save(t, {mpath!r}.encode(), {vpath!r}.encode())
"""
        env = dict(os.environ, MALLOC_PERTURB_="255", GLIBC_TUNABLES="glibc.malloc.tcache_count=0")
        subprocess.check_call([sys.executable, "-c", code], stdout=subprocess.DEVNULL, env=env)
        rows = np.frombuffer(open(mpath, "rb").read(), dtype="<i4").reshape(-1, 3).copy()
        freq = parse_vocab(open(vpath, "rb").read(), token_cstrings(rows))
    return rows, freq


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    with open(os.path.join(GOLD, "train_runs.txt"), "wb") as f:
        f.write(runs_text())
    index = []
    for name, rec, cfg in RECIPES:
        text = corpus_bytes(rec)
        rows, freq = run_reference(text, cfg)
        with open(os.path.join(GOLD, "train_%s.bin" % name), "wb") as f:
            f.write(rows.astype("<i4").tobytes())
        np.save(os.path.join(GOLD, "train_%s.freq.npy" % name), freq)
        index.append({"name": name, "corpus": rec, "config": list(cfg), "merges": int(len(rows)),
                      "corpus_bytes": len(text)})
        print(name, len(text), "bytes ->", len(rows), "merges")
    with open(os.path.join(GOLD, "train_index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
