"""GPU trainer (include/shredword_train.h) against the trainer oracle and the reference trainer's
own outputs (tests/golden/train_*): merges and final token frequencies, bit for bit."""
import json
import os

import numpy as np
import pytest

import oracle
import shredword_amd as sa
from test_train_oracle import INDEX, golden, recipe_text

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["default", "host_load", "full_scan"])
@pytest.mark.parametrize("entry", INDEX, ids=[e["name"] for e in INDEX])
def test_gpu_trainer_matches_reference(entry, mode, monkeypatch):
    """Bit-exact with the reference trainer (merges and final token frequencies): the corpus
    loaded on the device and every merge over its pair's word lists (the default); loaded by the
    host threads (SW_TRAIN_HOST_LOAD=1, the path a 64-bit word-hash collision takes); every merge
    over all words' filters (SW_TRAIN_FULL_SCAN=1)."""
    monkeypatch.setenv("SW_TRAIN_HOST_LOAD", "1" if mode == "host_load" else "0")
    monkeypatch.setenv("SW_TRAIN_FULL_SCAN", "1" if mode == "full_scan" else "0")
    text = recipe_text(entry["corpus"])
    target, unk, cov, minf = entry["config"]
    t = sa.BPETrainer(target, unk, cov, minf)
    t.load_text(text)
    assert t.train() == entry["merges"]
    rows, freq = golden(entry["name"])
    np.testing.assert_array_equal(t.merges, rows)
    np.testing.assert_array_equal(t.token_freq, freq)
    st = t.stats
    assert st["merges"] == entry["merges"] and st["symbols"] > 0
    t.destroy()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_trainer_matches_oracle_random(seed):
    """Small random corpora over a tiny alphabet (many ties, runs, unk characters)."""
    rng = np.random.default_rng(seed)
    alphabet = np.frombuffer(b"aabbbcdde\xc3\xa9xy", dtype=np.uint8)
    words = [bytes(rng.choice(alphabet, size=int(rng.integers(1, 12)))) for _ in range(400)]
    text = b" ".join(words[int(i)] for i in rng.integers(0, len(words), size=5000))
    cfg = (256 + 300, int(rng.integers(0, 3)), 0.9, 2)
    exp_rows, exp_freq = oracle.train(text, *cfg)
    t = sa.BPETrainer(*cfg)
    t.load_text(text)
    assert t.train() == len(exp_rows)
    np.testing.assert_array_equal(t.merges, exp_rows)
    np.testing.assert_array_equal(t.token_freq, exp_freq)


def test_gpu_trainer_edges_and_save(tmp_path):
    t = sa.BPETrainer(300, 0, 0.995, 2)
    t.load_text(b"")
    assert t.train() == 0
    t.load_text(b"ab ab ab cd")
    assert t.train() == 1
    assert t.merges.tolist() == [[97, 98, 256]]
    with pytest.raises(sa._lib.ShredwordError):
        t.load_text(b"a\0b")
    with pytest.raises(IOError):
        t.load_corpus(str(tmp_path / "missing.txt"))
    # file round trip: the same corpus from a file, saved model rows and vocab lines
    text = recipe_text(INDEX[3]["corpus"])
    p = tmp_path / "c.txt"
    p.write_bytes(text)
    target, unk, cov, minf = INDEX[3]["config"]
    t2 = sa.BPETrainer(target, unk, cov, minf)
    t2.load_corpus(str(p))
    n = t2.train()
    t2.save(str(tmp_path / "m.bin"), str(tmp_path / "v.txt"))
    rows = np.frombuffer((tmp_path / "m.bin").read_bytes(), dtype="<i4").reshape(-1, 3)
    np.testing.assert_array_equal(rows, golden(INDEX[3]["name"])[0])
    raw = (tmp_path / "v.txt").read_bytes()
    assert raw.count(b"\n") == 256 + n + 1  # one line per id, plus the token "\n" itself
    assert raw.endswith(b" %d\n" % int(t2.token_freq[-1]))
    # the trained merges encode through the GPU encoder like the oracle's encode does
    tok = t2.tokenizer()
    ids = tok.encode("aab ab ba xyz")
    assert tok.decode(ids) == "aab ab ba xyz"


def test_gpu_trainer_negative_unk_matches_oracle():
    """unk_id -1 (the reference's default in docs): unk symbols never pair in the count, but the
    merge deltas of their neighbours use the reference's change key, where a second member of -1
    sign-extends over the whole key (bpe.cpp:456-467, restated by both); token frequencies skip
    the negative id (bpe.cpp:709 would write freq[-1])."""
    rng = np.random.default_rng(9)
    alphabet = np.frombuffer(b"aaabbbcccdxyzQW!", dtype=np.uint8)
    words = [bytes(rng.choice(alphabet, size=int(rng.integers(2, 9)))) for _ in range(300)]
    text = b" ".join(words[int(i)] for i in rng.integers(0, len(words), size=8000))
    cfg = (256 + 200, -1, 0.7, 2)
    exp_rows, exp_freq = oracle.train(text, *cfg)
    t = sa.BPETrainer(*cfg)
    t.load_text(text)
    assert t.train() == len(exp_rows) > 0
    np.testing.assert_array_equal(t.merges, exp_rows)
    np.testing.assert_array_equal(t.token_freq, exp_freq)
    # save and tokenizer() with members that are the (negative) UNK id: a negative member renders
    # as the empty string, and tokenizer() leaves such merges out (no byte sequence reaches them)
    neg = [(int(a), int(b)) for a, b, _ in exp_rows if a < 0 or b < 0]
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        t.save(d + "/m.model", d + "/m.vocab")
        rows = np.fromfile(d + "/m.model", dtype=np.int32).reshape(-1, 3)
        np.testing.assert_array_equal(rows, exp_rows)
        vocab = open(d + "/m.vocab", "rb").read()
        assert vocab.endswith(b"\n") and vocab.count(b"\n") == 256 + len(exp_rows) + 1  # (+1: byte 10's own)
    tok = t.tokenizer()
    assert all(a >= 0 and b >= 0 for a, b in tok.merges)
    assert len(tok.merges) <= len(exp_rows) - len(neg)
    sample = b" ".join(words[:50]).decode()
    assert tok.decode(tok.encode(sample)) == sample
    tok.close()


def test_tokenizer_train():
    """Tokenizer.train (BaseTokenizer.train, abstract in the reference, base.py:107) drives the
    GPU trainer: the merges are the trainer's (equal to the oracle's), the vocabulary follows,
    and the trained tokenizer round-trips text, special tokens kept."""
    rng = np.random.default_rng(5)
    words = ["".join(rng.choice(list("abcdeé "), size=rng.integers(1, 9))) for _ in range(3000)]
    text = " ".join(words) + "\n"
    tok = sa.Tokenizer(device=0)
    tok.special_tokens = {"<|end|>": 100000}
    n = tok.train(text, 256 + 120, min_pair_freq=2, character_coverage=0.9999, unk_id=-1)
    assert 0 < n <= 120 and len(tok.merges) <= n
    exp_rows, _ = oracle.train(text.encode("utf-8"), 256 + 120, -1, 0.9999, 2)
    assert n == len(exp_rows)
    made, exp = set(range(256)), []
    for a, b, v in exp_rows.tolist():  # (merges built on the negative UNK id left out)
        if a in made and b in made:
            exp.append((a, b, v))
            made.add(v)
    assert [(a, b, v) for (a, b), v in tok.merges.items()] == exp
    for (a, b), v in tok.merges.items():
        assert tok.vocab[v] == tok.vocab[a] + tok.vocab[b]
    assert tok.special_tokens == {"<|end|>": 100000}
    s = "abc dé ea<|end|> bad"
    assert tok.decode(tok.encode(s)) == s
    assert len(tok.encode("abcde abcde")) < len("abcde abcde".encode("utf-8"))
