#!/usr/bin/env python3
"""Pin the oracle at scale: digests of the REFERENCE's encode of >= 16 MB of each bench corpus.

CONTAINER-ONLY test infrastructure (needs /root/reference, read-only).  The encode loop is the
one make_golden.py composes from the reference's own primitives, imported by file path from
/root/reference/shredword/base.py (apply_regex base.py:38-58, get_stats base.py:10-20, merge
base.py:22-36).  Inputs are prefixes of the exact batches bench.py times (corpus.synth with the
bench seed; a prefix of K strings does not depend on how many strings are generated).  Only
data is committed: per block of strings, the token count and the sha256 of the ids as
little-endian int32 -- tests/golden/scale_digests.json, checked against the oracle by
tests/test_oracle_golden.py (and through the oracle, the GPU at full size by
tests/test_gpu_fullsize.py).

    python oracle/make_golden_scale.py [--mb 16] [--procs 8]
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

import make_golden as mg  # noqa: E402  (the reference primitives, imported by path there)
from shredword_amd import corpus  # noqa: E402  (synthetic inputs only)

BENCH_SEED = 1_000_003
BLOCK = 256  # strings per digest block
CONFIGS = {
    # name: (corpus kind, mean length, model, pattern) -- bench.py's C2 and C5 batches
    "c2_mixed_bl32k_cl100k": (corpus.MIXED, 1074, "bl32k", "cl100k"),
    "c5_stress_bl50k_cl100k": (corpus.STRESS, 600, "bl50k", "cl100k"),
    "c2_mixed_bl32k_gpt2": (corpus.MIXED, 1074, "bl32k", "gpt2"),
    # round 4: the low-repetition corpus (bench.py --corpus entropy)
    "entropy_bl32k_cl100k": (corpus.ENTROPY, 1074, "bl32k", "cl100k"),
}

_MERGES = {}


def _block(args):
    model, pattern, texts = args
    if model not in _MERGES:
        _MERGES[model] = mg.load_merges(model)
    ids = []
    for t in texts:
        ids.extend(mg.ref_encode(t, _MERGES[model], pattern))
    a = np.asarray(ids, dtype="<i4")
    return len(ids), hashlib.sha256(a.tobytes()).hexdigest()


def prefix(kind, mean, min_bytes):
    n = 1024
    while True:
        buf, off = corpus.synth(BENCH_SEED, kind, n, mean, n_threads=8)
        if int(off[-1]) >= min_bytes:
            k = int(np.searchsorted(off, min_bytes, side="left"))
            k = ((k + BLOCK - 1) // BLOCK) * BLOCK  # whole blocks
            if k <= n:
                return buf[:int(off[k])], off[:k + 1]
        n *= 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=16.0)
    ap.add_argument("--gpt2-mb", type=float, default=4.0)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--only", default=None, help="regenerate this config only, keeping the others' digests")
    args = ap.parse_args()
    out = {"reference": mg.REF_BASE, "seed": BENCH_SEED, "block_strings": BLOCK, "configs": {}}
    path = os.path.join(mg.GOLD, "scale_digests.json")
    if args.only:
        with open(path) as f:
            out = json.load(f)
    with mp.get_context("fork").Pool(args.procs) as pool:
        for name, (kind, mean, model, pattern) in CONFIGS.items():
            if args.only and name != args.only:
                continue
            mb = args.gpt2_mb if pattern == "gpt2" else args.mb
            buf, off = prefix(kind, mean, int(mb * 1e6))
            data = bytes(buf)
            n = len(off) - 1
            jobs = []
            for b0 in range(0, n, BLOCK):
                texts = [data[off[s]:off[s + 1]].decode("utf-8") for s in range(b0, min(n, b0 + BLOCK))]
                jobs.append((model, pattern, texts))
            t = time.time()
            blocks = pool.map(_block, jobs, chunksize=1)
            out["configs"][name] = {"kind": int(kind), "mean_len": mean, "model": model + ".model",
                                    "pattern": pattern, "n_strings": n, "n_bytes": int(off[-1]),
                                    "n_tokens": sum(c for c, _ in blocks), "blocks": [[c, h] for c, h in blocks]}
            print("%s: %d strings, %.1f MB, %d tokens, %.0f s" % (name, n, off[-1] / 1e6,
                                                                    out["configs"][name]["n_tokens"], time.time() - t),
                  flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
