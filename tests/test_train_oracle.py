"""The trainer oracle (oracle/sw_train_oracle.c) against the reference trainer's own outputs
(tests/golden/train_*, made by oracle/make_train_golden.py from the reference sources): merge
rows and final token frequencies, bit for bit, on five recipes (CPU)."""
import json
import os

import numpy as np
import pytest

import oracle
from shredword_amd import corpus

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(GOLD, "train_index.json")))
KINDS = {"ascii": corpus.ASCII, "mixed": corpus.MIXED, "stress": corpus.STRESS}


def recipe_text(rec):
    if "file" in rec:
        return open(os.path.join(GOLD, rec["file"]), "rb").read()
    buf, _ = corpus.synth(rec["seed"], KINDS[rec["kind"]], rec["strings"], rec["mean"])
    return bytes(buf).replace(b"\0", b" ")


def golden(name):
    rows = np.frombuffer(open(os.path.join(GOLD, "train_%s.bin" % name), "rb").read(), dtype="<i4").reshape(-1, 3)
    return rows, np.load(os.path.join(GOLD, "train_%s.freq.npy" % name))


@pytest.mark.parametrize("entry", INDEX, ids=[e["name"] for e in INDEX])
def test_oracle_trainer_matches_reference(entry):
    text = recipe_text(entry["corpus"])
    assert len(text) == entry["corpus_bytes"]
    rows, freq = oracle.train(text, *entry["config"])
    exp_rows, exp_freq = golden(entry["name"])
    np.testing.assert_array_equal(rows, exp_rows)
    np.testing.assert_array_equal(freq, exp_freq)


def test_oracle_trainer_edges():
    assert len(oracle.train(b"", 300, 0, 0.995, 2)[0]) == 0
    assert len(oracle.train(b"ab ab ab", 256, 0, 0.995, 2)[0]) == 0          # no merges asked
    rows, freq = oracle.train(b"ab ab ab cd", 300, 0, 0.9999, 2)
    assert rows.tolist() == [[97, 98, 256]]                                   # (c, d) is below min_pair_freq
    assert freq[256] == 3 and freq[99] == 1 and freq[97] == 0
    with pytest.raises(ValueError):
        oracle.train(b"a\0b", 300, 0, 0.995, 2)                               # NUL bytes are rejected
