"""Pin the oracle (oracle/sw_oracle.c) to the golden vectors generated from the reference's own
primitives (oracle/make_golden.py).  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLD, PATTERNS, golden_index, load_fixture, load_model_merges

FIXTURES = golden_index()["fixtures"]


@pytest.mark.parametrize("entry", FIXTURES, ids=[e["file"] for e in FIXTURES])
def test_oracle_matches_reference_encode(entry):
    fx = load_fixture(entry)
    m = oracle.OracleModel(load_model_merges(entry["model"]))
    ids, off = m.encode_batch(fx["bytes"], fx["off"], PATTERNS[entry["pattern"]], n_threads=4)
    np.testing.assert_array_equal(off, fx["ids_off"])
    np.testing.assert_array_equal(ids, fx["ids"])


def test_oracle_threads_identical():
    entry = FIXTURES[1]
    fx = load_fixture(entry)
    m = oracle.OracleModel(load_model_merges(entry["model"]))
    a, ao = m.encode_batch(fx["bytes"], fx["off"], 0, n_threads=1)
    b, bo = m.encode_batch(fx["bytes"], fx["off"], 0, n_threads=7)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(ao, bo)


@pytest.mark.parametrize("pat", ["cl100k", "gpt2"])
def test_oracle_presplit_matches_reference(primitives, pat):
    for case in primitives["apply_regex_" + pat]:
        t = case["text"]
        data = t.encode("utf-8")
        st = oracle.presplit(data, PATTERNS[pat])
        ends = st[1:] + [len(data)]
        got = [data[a:e].decode("utf-8") for a, e in zip(st, ends)]
        assert got == case["chunks"], t


def test_oracle_primitive_kats(primitives):
    # merge(): the oracle's chunk loop on a table with one pair reproduces merge's outputs
    for case in primitives["merge"]:
        a, b = case["pair"]
        if any(x > 255 for x in case["ids"]) or case["idx"] < 256:
            continue
        m = oracle.OracleModel({(a, b): case["idx"]})
        data = bytes(case["ids"])
        # one merge step only applies when the pair is the sole merge; the full loop may merge
        # again on the new ids, which a one-pair table with idx > 255 never does
        assert m.encode_chunk(data) == case["out"]


SCALE = os.path.join(GOLD, "scale_digests.json")


@pytest.mark.parametrize("name", sorted(json.load(open(SCALE))["configs"]) if os.path.exists(SCALE) else [])
def test_oracle_matches_reference_at_scale(name):
    """The oracle on >= 16 MB prefixes of the bench's own C2 / C5 batches (4 MB with the GPT-2
    pattern) against digests of the REFERENCE's encode of the same strings (oracle/
    make_golden_scale.py: per block of strings, the token count and the sha256 of the ids)."""
    from shredword_amd import corpus
    g = json.load(open(SCALE))
    cfg = g["configs"][name]
    n = cfg["n_strings"]
    buf, off = corpus.synth(g["seed"], cfg["kind"], n, cfg["mean_len"], n_threads=8)
    assert int(off[-1]) == cfg["n_bytes"]
    m = oracle.OracleModel(load_model_merges(cfg["model"]))
    ids, ids_off = m.encode_batch(buf, off, PATTERNS[cfg["pattern"]], n_threads=8)
    assert len(ids) == cfg["n_tokens"]
    B = g["block_strings"]
    for k, (cnt, digest) in enumerate(cfg["blocks"]):
        s0, s1 = k * B, min(n, (k + 1) * B)
        blk = np.ascontiguousarray(ids[ids_off[s0]:ids_off[s1]], dtype="<i4")
        assert len(blk) == cnt, "block %d: %d ids, the reference %d" % (k, len(blk), cnt)
        assert hashlib.sha256(blk.tobytes()).hexdigest() == digest, "block %d (strings %d..%d)" % (k, s0, s1)


@pytest.mark.parametrize("model", ["toy500.model", "bl32k.model", "bl50k.model"])
def test_oracle_heap_form_equals_reference_loop(model):
    """The oracle's O(n log n) form for long chunks of well-formed tables (orc_encode_chunk_heap)
    gives exactly the reference loop's ids (orc_encode_chunk_naive, base.py:10-36 step by step)
    on long chunks of every kind: letter runs, (a, a) runs, whitespace runs, mixed text, raw bytes."""
    import random

    m = oracle.OracleModel(load_model_merges(model))
    assert m.well_formed
    rng = random.Random(21)
    cases = []
    for n in (256, 300, 700, 1500, 4096):
        cases.append(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(n)))
        cases.append(bytes(rng.choice(b"etaoin shrdlu") for _ in range(n)))
        cases.append(bytes([rng.choice(b"ab")]) * n)
        cases.append(b"".join(bytes([c]) * rng.randint(1, 40) for c in rng.choices(b"a ze\n", k=n))[:n])
        cases.append(bytes(rng.randrange(256) for _ in range(n)))
        cases.append(("Hello world, 中文字符 😀 " * (n // 20 + 1)).encode()[:n])
    for c in cases:
        assert m.encode_chunk(c, "heap") == m.encode_chunk(c, "naive"), (model, len(c), c[:40])
        assert m.encode_chunk(c) == m.encode_chunk(c, "naive")
