"""Special tokens (E1) on the host: the occurrence finder (sw_find_specials_host), the host
pre-split with occurrences (sw_presplit_host_specials) and the corpus splicer -- CPU only.

The reference stores `special_tokens` (shredword/base.py:103, saved/loaded at :120-121 /
:142-144) but defines no split; the build's rule is minbpe's: leftmost occurrence first, the
first special in dict order at one position.  The finder is checked against a plain restatement
of that rule (`split_ref`, the same one the oracle's orc_encode_with_specials implements), the
pre-split against the oracle's per-piece pre-split."""
import random

import numpy as np
import pytest

from shredword_amd import _lib, corpus
from conftest import ROOT  # noqa: F401  (sys.path set-up)

import oracle


def split_ref(text, specials):
    """(pos, len, id) of the occurrences in bytes `text`: at each position the first special in
    dict order that matches; the scan resumes after an occurrence."""
    out, i = [], 0
    names = [(s.encode("utf-8"), v) for s, v in specials.items() if s]
    while i < len(text):
        for b, v in names:
            if text.startswith(b, i):
                out.append((i, len(b), v))
                i += len(b)
                break
        else:
            i += 1
    return out


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


def found(datas, specials, n_threads=0):
    buf, off = pack(datas)
    pos, ln, ids = corpus.find_specials(buf, off, specials, n_threads=n_threads)
    return list(zip(pos.tolist(), ln.tolist(), ids.tolist())), buf, off


def test_rule_leftmost_then_dict_order():
    sp = {"<a>": 300, "<a><b>": 301, "<b>": 302}
    got, _, _ = found([b"x<a><b>y<b>"], sp)
    assert got == [(1, 3, 300), (4, 3, 302), (8, 3, 302)]
    sp = {"<a><b>": 301, "<a>": 300}
    got, _, _ = found([b"x<a><b>y<a>"], sp)
    assert got == [(1, 6, 301), (8, 3, 300)]
    got, _, _ = found([b"x<a>"], {})
    assert got == []
    # occurrences never cross strings; positions are batch-relative
    got, _, _ = found([b"ab<", b"a>", b"<a>"], {"<a>": 7})
    assert got == [(5, 3, 7)]
    # an empty special never matches
    got, _, _ = found([b"abc"], {"": 5, "b": 6})
    assert got == [(1, 1, 6)]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_finder_matches_rule_fuzz(seed):
    rng = random.Random(seed)
    specials = {"<|endoftext|>": 50256, "<|fim|>": 50257, "<|": 50258, "|>": 50259, "ab": 600, "a": 601,
                "中": 602, "\U0001f600x": 603}
    alphabet = ["a", "b", "ab", "<", "|", ">", "<|", "|>", "<|fim|>", "<|endoftext|>", " ", "\n", "中",
                "\U0001f600", "x", "é"]
    texts = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 60))).encode() for _ in range(400)]
    for nt in (1, 4):
        got, _, off = found(texts, specials, n_threads=nt)
        exp = []
        for s, t in enumerate(texts):
            exp += [(int(off[s]) + p, ln, v) for p, ln, v in split_ref(t, specials)]
        assert got == exp
    # several distinct first bytes and one (the memchr path)
    got1, _, off = found(texts, {"<|fim|>": 1, "<|endoftext|>": 2})
    exp1 = []
    for s, t in enumerate(texts):
        exp1 += [(int(off[s]) + p, ln, v) for p, ln, v in split_ref(t, {"<|fim|>": 1, "<|endoftext|>": 2})]
    assert got1 == exp1


@pytest.mark.parametrize("pattern", [_lib.SW_PAT_CL100K, _lib.SW_PAT_GPT2, _lib.SW_PAT_NONE])
def test_presplit_with_specials_matches_oracle_pieces(pattern):
    rng = random.Random(pattern + 11)
    specials = {"<|endoftext|>": 50256, "<|fim|>": 50257, " x": 50258}
    alphabet = ["word", " ", "  ", "\n", "123", "4567", "'s", "'LL", "!!", " <", "|", "<|fim|>", "<|endoftext|>",
                " x", "中文", "\U0001f642", "été", "\t", "\r\n"]
    texts = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 40))).encode() for _ in range(600)]
    buf, off = pack(texts)
    pos, ln, ids = corpus.find_specials(buf, off, specials)
    bits, cnt = corpus.presplit_specials(buf, off, pos, ln, pattern)
    exp = np.zeros_like(bits)
    n_exp = 0
    for s, t in enumerate(texts):
        base = int(off[s])
        seg = 0
        for p, L, _ in split_ref(t, specials) + [(len(t), 0, None)]:
            piece = t[seg:p]
            for c in oracle.presplit(piece, pattern):
                q = base + seg + c
                exp[q >> 6] |= np.uint64(1 << (q & 63))
                n_exp += 1
            if L:
                q = base + p
                exp[q >> 6] |= np.uint64(1 << (q & 63))
                n_exp += 1
            seg = p + L
    assert cnt == n_exp
    np.testing.assert_array_equal(bits, exp)


def test_splice_specials_deterministic_and_valid():
    buf, off = corpus.synth(3, corpus.MIXED, 500, 700, n_threads=1)
    sp = {"<|endoftext|>": 50256, "<|fim_prefix|>": 50257}
    a, ao = corpus.splice_specials(buf, off, sp, per_kib=2.0, end_special=0, n_threads=1)
    b, bo = corpus.splice_specials(buf, off, sp, per_kib=2.0, end_special=0, n_threads=7)
    assert (ao == bo).all() and (a == b).all()
    bytes(a).decode("utf-8")
    for s in range(len(off) - 1):  # every string ends with the separator and keeps its text in order
        t = bytes(a[ao[s]:ao[s + 1]])
        assert t.endswith(b"<|endoftext|>")
        assert t.replace(b"<|endoftext|>", b"").replace(b"<|fim_prefix|>", b"") == bytes(buf[off[s]:off[s + 1]])
    pos, ln, ids = corpus.find_specials(a, ao, sp)
    assert len(pos) >= len(off) - 1


def test_entropy_corpus_deterministic_and_valid():
    a, ao = corpus.synth(5, corpus.ENTROPY, 300, 600, n_threads=1)
    b, bo = corpus.synth(5, corpus.ENTROPY, 300, 600, n_threads=5)
    assert (ao == bo).all() and (a == b).all()
    text = bytes(a).decode("utf-8")
    scripts = {"cyrillic": any("Ѐ" <= ch <= "ӿ" for ch in text), "greek": any("Ͱ" <= ch <= "Ͽ" for ch in text),
               "cjk": any("一" <= ch <= "鿿" for ch in text), "hangul": any("가" <= ch <= "힣" for ch in text),
               "devanagari": any("ऀ" <= ch <= "ॿ" for ch in text)}
    assert all(scripts.values()), scripts


def test_bad_arguments():
    L = _lib.lib()
    assert L.sw_find_specials_host(None, None, -1, None, None, None, None, 0, 1) == _lib.SW_ERR_ARG
    buf, off = pack([b"abcab"])
    pos = np.array([3, 1], dtype=np.int64)  # (not ascending)
    ln = np.array([1, 1], dtype=np.int32)
    bits = np.zeros(1, dtype=np.uint64)
    assert L.sw_presplit_host_specials(_lib.ptr(buf, __import__("ctypes").c_uint8),
                                       _lib.ptr(off, __import__("ctypes").c_int64), 1, 0,
                                       _lib.ptr(pos, __import__("ctypes").c_int64),
                                       _lib.ptr(ln, __import__("ctypes").c_int32), 2,
                                       _lib.ptr(bits, __import__("ctypes").c_uint64), 1) == _lib.SW_ERR_ARG
    with pytest.raises(ValueError):
        _lib.specials_struct({"<x>": -1})
