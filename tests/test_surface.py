"""The Python surface (shredword/base.py mirror) and the native host pre-split, against the
reference's golden vectors.  CPU only."""
import os
import random

import numpy as np
import pytest
import regex

import oracle
import shredword_amd as sa
from shredword_amd import base as sb
from shredword_amd import corpus
from conftest import GOLD, PATTERNS, load_model_merges


def test_get_stats_kat(primitives):
    for case in primitives["get_stats"]:
        got = [[a, b, c] for (a, b), c in sa.get_stats(case["ids"]).items()]
        assert got == case["stats"]


def test_merge_kat(primitives):
    for case in primitives["merge"]:
        assert sa.merge(case["ids"], tuple(case["pair"]), case["idx"]) == case["out"]


@pytest.mark.parametrize("pat", ["cl100k", "gpt2"])
def test_apply_regex_native_matches_reference(primitives, pat):
    p = "" if pat == "cl100k" else sa.GPT2_PATTERN
    for case in primitives["apply_regex_" + pat]:
        assert sa.apply_regex(case["text"], p) == case["chunks"], case["text"]


def test_build_vocab_and_render(primitives):
    bv = primitives["build_vocab"]
    m = {(a, b): i for a, b, i in bv["merges"]}
    sp = {k: i for k, i in bv["special"]}
    got = sa.build_vocab(m, sp)
    assert [[i, list(b)] for i, b in got.items()] == bv["vocab"]
    for case in primitives["render_token"]:
        assert sa.render_token(bytes(case["bytes"])) == case["out"]


def test_load_save_match_reference(primitives, tmp_path):
    kat = primitives["load"]
    path = tmp_path / "x.model"
    path.write_text(kat["text"], encoding="utf-8")
    t = sa.BaseTokenizer()
    t.load(str(path))
    assert t.pattern == kat["pattern"]
    assert [[a, b, i] for (a, b), i in t.merges.items()] == kat["merges"]
    assert [[k, i] for k, i in t.special_tokens.items()] == kat["special"]
    assert [[i, list(b)] for i, b in t.vocab.items()] == kat["vocab"]
    t.save(str(tmp_path / "out"))
    assert (tmp_path / "out.model").read_text(encoding="utf-8") == primitives["save"]["model"]
    assert (tmp_path / "out.vocab").read_text(encoding="utf-8") == primitives["save"]["vocab"]


def test_load_error_behaviour(primitives, tmp_path):
    kat = primitives["load_error"]
    path = tmp_path / "bad.model"
    path.write_text(kat["text"])
    if kat["error"] is None:
        sa.BaseTokenizer().load(str(path))
    else:
        with pytest.raises(Exception) as ei:
            sa.BaseTokenizer().load(str(path))
        assert type(ei.value).__name__ == kat["error"]
    with pytest.raises(AssertionError):
        sa.BaseTokenizer().load(str(tmp_path / "x.txt"))


def test_load_binary_trainer_format():
    t1, t2 = sa.BaseTokenizer(), sa.BaseTokenizer()
    t1.load(os.path.join(GOLD, "toy500.model"))
    t2.load_binary(os.path.join(GOLD, "toy500.bin"))
    assert t1.merges == t2.merges
    assert t1.vocab == t2.vocab


def _bits_to_starts(bits, n):
    return np.flatnonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:n]).tolist()


@pytest.mark.parametrize("kind", [corpus.MIXED, corpus.STRESS, corpus.ASCII])
@pytest.mark.parametrize("pat", [0, 1])
def test_host_presplit_matches_oracle_on_corpus(kind, pat):
    buf, off = corpus.synth(77 + kind, kind, 600, 700)
    bits, cnt = corpus.presplit(buf, off, pat, n_threads=4)
    got = _bits_to_starts(bits, int(off[-1]))
    exp = []
    data = bytes(buf)
    for s in range(len(off) - 1):
        a = int(off[s])
        exp.extend(a + x for x in oracle.presplit(data[a:int(off[s + 1])], pat))
    assert cnt == len(exp)
    assert got == exp


def test_host_presplit_random_unicode_vs_regex():
    rng = random.Random(3)
    pool = [chr(c) for c in list(range(0x20, 0x7F)) + [9, 10, 13, 11, 12, 0x1C, 0x85, 0xA0, 0x17F, 0x1680, 0x2000, 0x2028,
                                                      0x3000, 0x4E00, 0x1F600, 0xE9, 0x301, 0x660, 0x1C89, 0x10EC2]]
    for _ in range(1500):
        t = "".join(rng.choice(pool) for _ in range(rng.randint(0, 30)))
        assert sa.apply_regex(t) == regex.findall(sb.CL100K_PATTERN, t)
        assert sa.apply_regex(t, sa.GPT2_PATTERN) == regex.findall(sa.GPT2_PATTERN, t)


def test_host_presplit_invalid_utf8_is_a_tiling():
    # bytes no Python str can produce: every byte still belongs to exactly one chunk,
    # and host and oracle agree
    rng = random.Random(9)
    for _ in range(300):
        data = bytes(rng.choice(b"ab \n\x80\xff\xc3\xa9\xe4\xb8") for _ in range(rng.randint(1, 40)))
        for pat in (0, 1):
            assert sb.split_chunks(data, pat) == oracle.presplit(data, pat)


def test_pattern_selection():
    assert sb.pattern_id("") == 0
    assert sb.pattern_id(sb.CL100K_PATTERN) == 0
    assert sb.pattern_id(sb.GPT2_PATTERN) == 1
    assert sb.pattern_id(sb.GPT2_PATTERN_ALT) == 1
    assert sb.pattern_id(2) == 2
    # any other pattern string: cl100k, as the reference's apply_regex (base.py:56) does
    pattern3 = r"""'s|'t|'re|'ve|'m|'ll|'d|[\w']+|[^\s\w\d]+|\s+(?!\S)|\s+"""
    with pytest.warns(UserWarning, match="cl100k"):
        assert sb.pattern_id(pattern3) == 0
    for bad in (7, -1):
        with pytest.raises(ValueError):
            sb.pattern_id(bad)
    with pytest.raises(TypeError):
        sb.pattern_id(None)


def test_tracked_merges_and_vocab():
    # edits of every kind bump the version the device table is keyed on
    t = sa.Tokenizer(device=0)
    seen = [t.merges.version]
    t.merges[(97, 98)] = 256
    seen.append(t.merges.version)
    t.merges |= {(99, 100): 257}  # (__ior__, then the property setter)
    seen.append(t.merges.version)
    d = t.merges
    d |= {(1, 2): 259}  # __ior__ alone
    seen.append(t.merges.version)
    t.merges.update({(256, 257): 258})
    seen.append(t.merges.version)
    assert all(a < b for a, b in zip(seen, seen[1:])), seen
    assert isinstance(t.merges, type(t.merges)) and t.merges[(99, 100)] == 257
    # a same-size replacement rebuilds the vocabulary decode uses
    t.merges = {(97, 98): 256}
    assert t._vocab_now()[256] == b"ab"
    t.merges = {(99, 100): 256}
    assert t._vocab_now()[256] == b"cd"
    t.merges[(99, 100)] = 300  # in-place value change
    assert t._vocab_now()[300] == b"cd"
    t.special_tokens["<|x|>"] = 400
    assert t._vocab_now()[400] == b"<|x|>"
    # a vocab assigned directly is used as given until merges/specials change
    ver = t.vocab.version
    t.vocab = dict(t.vocab, **{})
    assert t.vocab.version == ver + 1
    t.vocab[5] = b"zz"
    assert t._vocab_now()[5] == b"zz" and t.vocab.version == ver + 2


def test_corpus_deterministic_across_threads():
    a, ao = corpus.synth(5, corpus.MIXED, 300, 500, n_threads=1)
    b, bo = corpus.synth(5, corpus.MIXED, 300, 500, n_threads=5)
    assert (ao == bo).all() and (a == b).all()
    bytes(a).decode("utf-8")  # valid UTF-8 throughout
