"""Pin the oracle (oracle/sw_oracle.c) to the golden vectors generated from the reference's own
primitives (oracle/make_golden.py).  CPU only."""
import numpy as np
import pytest

import oracle
from conftest import PATTERNS, golden_index, load_fixture, load_model_merges

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
