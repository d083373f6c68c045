"""Parity of the HIP encode path with the reference semantics, on a gfx950 device.

Bit-exact comparisons (integer work): against the golden vectors produced by the reference's own
primitives (tests/golden), and against the oracle restatement (oracle/sw_oracle.c, itself pinned
to those vectors by test_oracle_golden.py) on seeded inputs and edge cases.  All calls go
through the C-ABI (shredword_amd -> libshredword_hip.so).
"""
import os
import random

import numpy as np
import pytest

import oracle
import shredword_amd as sa
from shredword_amd import _lib, corpus
from conftest import GOLD, PATTERNS, golden_index, load_fixture, load_model_merges

pytestmark = pytest.mark.gpu

FIXTURES = golden_index()["fixtures"]
PAT_STR = {"cl100k": "", "gpt2": sa.GPT2_PATTERN, "none": 2}


@pytest.fixture(scope="module", autouse=True)
def need_device():
    if _lib.lib().sw_device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu must run on the MI355X box")


_TOKS = {}


def tok_for(model, pattern="cl100k"):
    key = (model, pattern)
    if key not in _TOKS:
        t = sa.Tokenizer(device=0)
        t.merges = load_model_merges(model)
        _TOKS[key] = t
    t = _TOKS[key]
    t.pattern = PAT_STR[pattern]
    return t


def gpu_encode(t, buf, off):
    return t.encode_packed(buf, off)


def oracle_encode(merges, buf, off, pattern):
    return oracle.OracleModel(merges).encode_batch(buf, off, PATTERNS[pattern], n_threads=8)


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:max(int(off[-1]), 0)], off


def assert_same(got, exp):
    np.testing.assert_array_equal(got[1], exp[1])
    np.testing.assert_array_equal(got[0], exp[0])


@pytest.mark.parametrize("entry", FIXTURES, ids=[e["file"] for e in FIXTURES])
def test_golden_bit_exact(entry):
    fx = load_fixture(entry)
    t = tok_for(entry["model"], entry["pattern"])
    got = gpu_encode(t, fx["bytes"], fx["off"])
    assert_same(got, (fx["ids"], fx["ids_off"]))


@pytest.mark.parametrize("fork", [0, 1])
def test_merge_streams_option(fork):
    """The length buckets' merge kernels forked onto parallel streams (default) or one after
    another on the launch stream: the same ids as the reference-generated fixtures."""
    for entry in golden_index()["fixtures"]:
        fx = load_fixture(entry)
        t = sa.Tokenizer(device=0)
        t.merges = load_model_merges(entry["model"])
        t.pattern = PAT_STR[entry["pattern"]]
        _lib.check(_lib.lib().sw_encoder_set_option(t._encoder(), _lib.SW_OPT_MERGE_STREAMS, fork))
        assert_same(gpu_encode(t, fx["bytes"], fx["off"]), (fx["ids"], fx["ids_off"]))
        t.close()


def test_compaction_string_layouts():
    """Tile counts + scan + compaction (k_tile_count, k_compact): the reference-generated
    fixtures, then MIXED (20k strings, several per tile) and STRESS (4 KiB results) batches
    against the oracle, and tiny strings (many string starts per tile)."""
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges("bl32k.model")
    try:
        for entry in golden_index()["fixtures"]:
            if entry["model"] != "bl32k.model":
                continue
            fx = load_fixture(entry)
            t.pattern = PAT_STR[entry["pattern"]]
            assert_same(gpu_encode(t, fx["bytes"], fx["off"]), (fx["ids"], fx["ids_off"]))
        t.pattern = ""
        for seed, kind, n, mean in ((3, corpus.MIXED, 20000, 300), (4, corpus.STRESS, 3000, 600)):
            buf, off = corpus.synth(seed, kind, n, mean)
            assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, "cl100k"))
        rng = random.Random(5)
        buf, off = pack([bytes(rng.choice(b"ab ,.1") for _ in range(rng.randrange(0, 5))) for _ in range(50000)])
        assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, "cl100k"))
    finally:
        t.close()


@pytest.mark.parametrize("kernel", [1, 2, 3, 0])
def test_compaction_kernel_choice(kernel):
    """SW_OPT_COMPACT_KERNEL: the 6-wave (1024 staged ids a group), 7-wave (768) and 7-wave typed
    compaction kernels, forced and chosen per launch from the previous launch's ids per tile (0):
    a batch of many short ids per tile (its groups overflow the staging) after one of few and
    back, each against the oracle; other values are rejected."""
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges("bl32k.model")
    t.pattern = ""
    try:
        L = _lib.lib()
        assert L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_COMPACT_KERNEL, 4) != 0
        _lib.check(L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_COMPACT_KERNEL, kernel))
        rng = random.Random(11)
        dense = pack([bytes(rng.randrange(128, 256) for _ in range(rng.randrange(1, 600))) for _ in range(3000)])
        for buf, off in (corpus.synth(3, corpus.MIXED, 20000, 300), dense, corpus.synth(4, corpus.STRESS, 3000, 600),
                         dense):
            assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, "cl100k"))
    finally:
        t.close()


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("model", ["bl32k.model", "toy500.model", "wide"])
def test_staged_result_heads(mode, model):
    """SW_OPT_STAGED_HEADS: k_tile_count gathering each tile's result heads once and staging them over
    its reference list for k_compact (1: forced) against the gathers in k_compact (2) -- dense and
    own references, tiles over the staging's 512 heads (a one-byte-string batch of multi-token
    chunks), 16- and 32-bit heads (a table with ids over 16 bits), each == the oracle."""
    t = sa.Tokenizer(device=0)
    base = load_model_merges("bl32k.model" if model == "wide" else model)
    t.merges = ({(a if a < 256 else a + 70000, b if b < 256 else b + 70000): v + 70000 for (a, b), v in base.items()}
                if model == "wide" else base)
    t.pattern = ""
    try:
        L = _lib.lib()
        assert L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_STAGED_HEADS, 3) != 0
        _lib.check(L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_STAGED_HEADS, mode))
        rng = random.Random(12)
        many = pack([bytes(rng.choice(b"abcdefgh") for _ in range(rng.randrange(2, 5))) for _ in range(40000)])
        for buf, off in (corpus.synth(5, corpus.MIXED, 20000, 300), corpus.synth(6, corpus.ENTROPY, 8000, 500),
                         many, corpus.synth(7, corpus.STRESS, 3000, 600)):
            assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, "cl100k"))
    finally:
        t.close()


def test_tokenizer_encode_decode_surface():
    t = tok_for("bl32k.model")
    text = "Hello world's 12345 \n\n  x 中文 😀"
    ids = t.encode(text)
    assert ids == oracle.OracleModel(t.merges).encode_ordinary(text)
    assert t.decode(ids) == text
    assert t.encode_batch([text, "", text]) == [ids, [], ids]
    t.special_tokens = {"<|endoftext|>": 100257, "<|fim|>": 100258}
    s = "a<|endoftext|>b<|fim|><|endoftext|>"
    assert t.encode(s) == oracle.OracleModel(t.merges).encode_with_specials(s, t.special_tokens)
    assert t.encode(s, allowed_special="none") == oracle.OracleModel(t.merges).encode_ordinary(s)
    t.special_tokens = {}


def test_empty_inputs():
    t = tok_for("toy500.model")
    ids, off = gpu_encode(t, np.zeros(0, np.uint8), np.zeros(1, np.int64))
    assert len(ids) == 0 and off.tolist() == [0]
    ids, off = gpu_encode(t, np.zeros(0, np.uint8), np.zeros(5, np.int64))
    assert len(ids) == 0 and off.tolist() == [0] * 5
    buf, off = pack([b"", b"a", b"", b"", b"hello there", b""])
    assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, "cl100k"))


@pytest.mark.parametrize("model", ["toy500.model", "bl32k.model", "bl50k.model"])
def test_tile_boundaries_and_long_chunks(model):
    """Chunks that straddle the 2 KiB tiles, chunks longer than the per-lane limit (16 B), longer
    than a tile, and a 200 KB single chunk; (a,a) runs of every parity."""
    rng = random.Random(1)
    t = tok_for(model)
    datas = []
    for L in (1, 2, 15, 16, 17, 31, 63, 64, 65, 127, 2047, 2048, 2049, 4095, 4096, 4097, 9000, 200_000):
        datas.append(bytes(rng.choice(b"abcdefghij") for _ in range(L)))
        datas.append(b"a" * L)
        datas.append(b" " * L)
    for shift in range(0, 40):  # push word boundaries across the 2048-byte tile edges
        datas.append(b"x" * shift + b" hello world the of and" * 150)
    buf, off = pack(datas)
    assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, "cl100k"))


def test_self_pair_runs_exact():
    """(a,a) overlap rule of merge(): [a,a,a]->[X,a], [a,a,a,a]->[X,X] (base.py:29-35)."""
    merges = {(97, 97): 256, (256, 256): 257, (256, 97): 258, (257, 257): 259, (98, 98): 260}
    t = sa.Tokenizer()
    t.merges = merges
    datas = [b"a" * n for n in range(0, 300)] + [b"b" * n + b"a" * m for n in range(0, 20) for m in range(0, 20)]
    buf, off = pack(datas)
    t.pattern = 2
    assert_same(gpu_encode(t, buf, off), oracle_encode(merges, buf, off, "none"))


@pytest.mark.parametrize("seed", range(6))
def test_random_illformed_tables(seed):
    """Exactness must not depend on well-formedness: random pairs, duplicate values, values
    smaller than their pair members, ids > 255 referenced before they exist."""
    r = random.Random(seed)
    alpha = list(b"abcd ")
    ids = alpha + list(range(256, 256 + 40))
    merges = {}
    for _ in range(r.randint(5, 300)):
        merges[(r.choice(ids), r.choice(ids))] = r.randint(0, 300) if seed % 2 else r.randint(256, 295)
    datas = [bytes(r.choice(b"abcd ") for _ in range(r.randint(0, 120))) for _ in range(400)]
    datas.append(bytes(r.choice(b"abcd") for _ in range(5000)))
    buf, off = pack(datas)
    t = sa.Tokenizer()
    t.merges = merges
    for pat in ("none", "cl100k"):
        t.pattern = PAT_STR[pat]
        assert_same(gpu_encode(t, buf, off), oracle_encode(merges, buf, off, pat))


@pytest.mark.parametrize("seed", range(8))
def test_random_wellformed_tables(seed):
    """Random WELL-FORMED tables (every value new, >= 256 and larger than its pair's members)
    take the bit-mask merge loop with the ids in LDS (kernels.h lane_merge_lds_wf) in every
    merge bucket and in the long chunks' pieces and windows: a 3-letter alphabet with many (a, a)
    pairs (runs resolved left to right, base.py:29-35), chunks of every length 1..40 and a few
    long ones, against the oracle."""
    r = random.Random(100 + seed)
    alpha = list(b"abc")
    ids = list(alpha)
    merges = {}
    nxt = 256
    for _ in range(r.randint(20, 400)):
        a, b = r.choice(ids), r.choice(ids)
        if r.random() < 0.3:
            b = a  # (a, a) pairs
        if (a, b) in merges:
            continue
        merges[(a, b)] = nxt
        ids.append(nxt)
        nxt += 1
    datas = [bytes(r.choice(b"abc") for _ in range(n)) for n in range(0, 41) for _ in range(20)]
    datas += [bytes(r.choice(b"aab") for _ in range(r.randint(33, 3000))) for _ in range(20)]
    datas += [b"a" * n for n in range(1, 70)]
    buf, off = pack(datas)
    t = sa.Tokenizer()
    t.merges = merges
    L = _lib.lib()
    assert L.sw_encoder_get_info(t._encoder(), _lib.SW_INFO_IDS16) == 1
    assert L.sw_encoder_get_info(t._encoder(), _lib.SW_INFO_SPLIT) == 1
    t.pattern = PAT_STR["none"]
    assert_same(gpu_encode(t, buf, off), oracle_encode(merges, buf, off, "none"))


def test_wide_ids_table():
    """Ids > 65535 (e.g. vocabularies past 64k): the 16-byte-slot table path."""
    base = load_model_merges("bl32k.model")
    shift = lambda x: x if x < 256 else x + 70000  # noqa: E731
    merges = {(shift(a), shift(b)): shift(v) for (a, b), v in base.items()}
    fx = load_fixture(FIXTURES[1])
    t = sa.Tokenizer()
    t.merges = merges
    got = gpu_encode(t, fx["bytes"], fx["off"])
    exp_ids = np.where(fx["ids"] < 256, fx["ids"], fx["ids"] + 70000)
    assert_same(got, (exp_ids, fx["ids_off"]))


def test_invalid_utf8_bytes():
    """Invalid UTF-8 is BUILD-DEFINED: a Python str cannot carry invalid bytes into the
    reference's apply_regex (base.py:38-58), so nothing reference-side pins this case.  The
    build's rule: an invalid byte is a one-byte code point of class "other";
    the GPU pre-split and the oracle's follow it identically, which is all this checks."""
    rng = random.Random(4)
    datas = [bytes(rng.choice(b"ab \n\x80\xff\xc3\xa9\xe4\xb8\xf0\x9f") for _ in range(rng.randint(0, 80)))
             for _ in range(500)]
    buf, off = pack(datas)
    for model in ("toy500.model", "bl32k.model"):
        t = tok_for(model)
        for pat in ("cl100k", "gpt2"):
            t.pattern = PAT_STR[pat]
            assert_same(gpu_encode(t, buf, off), oracle_encode(t.merges, buf, off, pat))
        t.pattern = ""


@pytest.mark.parametrize("kind,model,pattern", [(corpus.MIXED, "bl32k.model", "cl100k"),
                                               (corpus.STRESS, "bl50k.model", "cl100k"),
                                               (corpus.MIXED, "bl32k.model", "gpt2")])
def test_large_corpus_vs_oracle(kind, model, pattern):
    """64 MB (MIXED) / 24 MB (STRESS) seeded corpora, bit-exact against the multithreaded oracle;
    the GPT-2 pattern's device pre-split at 64 MB too (checked against the oracle directly, not
    only against the host pre-split)."""
    n = 60000 if kind == corpus.MIXED else 40000
    buf, off = corpus.synth(99, kind, n, 1074 if kind == corpus.MIXED else 600)
    t = tok_for(model, pattern)
    got = gpu_encode(t, buf, off)
    assert_same(got, oracle_encode(t.merges, buf, off, pattern))


def test_device_api_with_torch_buffers():
    """sw_encode_device on torch-allocated HBM buffers and torch's stream."""
    import ctypes

    import torch
    buf, off = corpus.synth(7, corpus.MIXED, 3000, 1074)
    bits, _ = corpus.presplit(buf, off)
    t = tok_for("bl32k.model")
    exp = gpu_encode(t, buf, off)
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_bits = torch.from_numpy(bits.view(np.int64)).to(dev)
    d_out = torch.empty(len(buf), dtype=torch.int32, device=dev)
    d_oo = torch.empty(len(off), dtype=torch.int64, device=dev)
    n_tok = ctypes.c_int64()
    L = _lib.lib()
    _lib.check(L.sw_encode_device(t._encoder(), d_buf.data_ptr(), len(buf), d_off.data_ptr(), len(off) - 1,
                                  d_bits.data_ptr(), d_out.data_ptr(), d_oo.data_ptr(),
                                  torch.cuda.current_stream(dev).cuda_stream, ctypes.byref(n_tok)))
    torch.cuda.synchronize()
    assert n_tok.value == len(exp[0])
    np.testing.assert_array_equal(d_out[:n_tok.value].cpu().numpy(), exp[0])
    np.testing.assert_array_equal(d_oo.cpu().numpy(), exp[1])


@pytest.mark.parametrize("slots,fp_bits,exact", [
    (8, 0, 1), (8, 26, 0), (64, 0, 0), (1 << 12, 3, 1), (0, 26, 1), (0, 2, 0)])
def test_dedupe_table_pressure_and_collisions(slots, fp_bits, exact):
    """The batch-wide dedupe must never change a result: a table too small for the distinct
    chunks (fallback: chunks merge on their own), fingerprints cut to 0..3 bits (every probe
    decided by the byte comparison alone), exact keys on or off give the oracle's ids; so does
    dedupe switched off."""
    buf, off = corpus.synth(7, corpus.MIXED, 6000, 1074)
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    L, h = _lib.lib(), t._encoder()
    try:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_SLOTS, slots))
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_FP_BITS, fp_bits))
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_EXACT, exact))
        assert_same(gpu_encode(t, buf, off), exp)
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE, 0))
        assert_same(gpu_encode(t, buf, off), exp)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE, 1)
        L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_SLOTS, 0)
        L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_FP_BITS, 26)
        L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_EXACT, 1)


def test_dedupe_exact_key_prefix_collisions():
    """Chunks equal in their first 7 (or 14) bytes and length but not after (exact keys up to 7
    bytes, fingerprint keys beyond) must stay apart, each sharing only its own result, in a
    one-group table where they all meet."""
    rng = np.random.default_rng(11)
    stems = [" abcdefg", " qwertyu", " zxcvbnm", " abcdefghijklm", " abcdefghijklz"]
    words = [st + "".join(chr(0x61 + int(c)) for c in rng.integers(0, 26, size=k))
             for st in stems for k in (0, 1, 2, 3, 4, 7) for _ in range(6)]
    texts = ["".join(rng.choice(words, size=40)) for _ in range(300)]
    buf, off = pack([x.encode() for x in texts])
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    L, h = _lib.lib(), t._encoder()
    try:
        for slots in (8, 0):
            _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_SLOTS, slots))
            assert_same(gpu_encode(t, buf, off), exp)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_SLOTS, 0)


def test_dedupe_table_grows_and_clears_itself():
    """A low-repetition batch overflows the dedupe table the encoder starts with (~1 entry per 64
    input bytes): the launch after it grows the table, and no launch clears the table (the merge
    kernels empty the entries their chunks claimed) -- three launches of the same batch, each
    against the oracle, and another batch after them."""
    buf, off = corpus.synth(31, corpus.ENTROPY, 60000, 1074)
    buf2, off2 = corpus.synth(32, corpus.ENTROPY, 6000, 1074)
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    L, h = _lib.lib(), t._encoder()
    slots0 = None
    for rep in range(3):
        assert_same(gpu_encode(t, buf, off), exp)
        if rep == 0:
            slots0 = L.sw_encoder_get_info(h, _lib.SW_INFO_DEDUPE_SLOTS)
    grown = L.sw_encoder_get_info(h, _lib.SW_INFO_DEDUPE_SLOTS)
    assert grown > slots0
    # smaller launches after growth use (and clear) a prefix of the table sized for their bytes
    # (launch_dd_slots) and never grow it; the whole table again for the large batch after them
    buf3, off3 = corpus.synth(33, corpus.ENTROPY, 40, 900)
    for b, o in ((buf2, off2), (buf3, off3), (buf2, off2)):
        assert_same(gpu_encode(t, b, o), oracle_encode(t.merges, b, o, "cl100k"))
    assert L.sw_encoder_get_info(h, _lib.SW_INFO_DEDUPE_SLOTS) == grown
    assert_same(gpu_encode(t, buf, off), exp)


def test_dedupe_options_validated():
    t = tok_for("toy500.model")
    L, h = _lib.lib(), t._encoder()
    for opt, bad in ((_lib.SW_OPT_DEDUPE_SLOTS, 12), (_lib.SW_OPT_DEDUPE_SLOTS, 4), (_lib.SW_OPT_DEDUPE_FP_BITS, 27),
                     (99, 1)):
        assert L.sw_encoder_set_option(h, opt, bad) == _lib.SW_ERR_ARG


@pytest.mark.parametrize("fixture,model", [("enc_bl50k_stress.npz", "bl50k.model"), ("enc_bl32k_mixed.npz", "bl32k.model")])
def test_out_bits16_per_call(fixture, model):
    """sw_encode_device_ex out_bits 16 writes uint16 ids (the multi-GPU transport's width) -- the
    reference-generated ids' low 16 bits, ids >= 32768 included (bl50k) -- for that call only: a
    later sw_encode_device / Tokenizer.encode_device on the same handle writes int32 again (the
    former persistent SW_OPT_OUT_BITS is rejected); 16 bits is refused for a table with an id over
    16 bits; sw_encode_batch returns int32."""
    import ctypes

    import torch
    fx = np.load(os.path.join(GOLD, fixture))
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges(model)
    L, h = _lib.lib(), t._encoder()
    assert L.sw_encoder_set_option(h, _lib.SW_OPT_OUT_BITS, 16) == _lib.SW_ERR_ARG
    dev = torch.device("cuda", 0)
    d_buf, d_off = torch.from_numpy(fx["bytes"]).to(dev), torch.from_numpy(fx["off"]).to(dev)
    d_out = torch.full((len(fx["bytes"]) + 8,), -1, dtype=torch.int16, device=dev)
    d_oo = torch.empty(len(fx["off"]), dtype=torch.int64, device=dev)
    n_tok = ctypes.c_int64()
    ex = _lib.SwEncodeEx(None, 16, None, None, None, 0)
    _lib.check(L.sw_encode_device_ex(h, d_buf.data_ptr(), len(fx["bytes"]), d_off.data_ptr(), len(fx["off"]) - 1,
                                     ctypes.byref(ex), d_out.data_ptr(), d_oo.data_ptr(),
                                     torch.cuda.current_stream(dev).cuda_stream, ctypes.byref(n_tok)))
    n = n_tok.value
    assert n == len(fx["ids"])
    np.testing.assert_array_equal(d_out[:n].cpu().numpy().view(np.uint16).astype(np.int64), fx["ids"])
    assert int(d_out[n].item()) == -1  # (nothing written past the ids)
    np.testing.assert_array_equal(d_oo.cpu().numpy(), fx["ids_off"])
    # the next calls on the same handle: int32 again
    ids, off = t.encode_device(d_buf, d_off)
    assert ids.dtype == torch.int32
    np.testing.assert_array_equal(ids.cpu().numpy(), fx["ids"])
    ids16, _ = t.encode_device(d_buf, d_off, out_bits=16)
    np.testing.assert_array_equal(ids16.cpu().numpy().view(np.uint16).astype(np.int64), fx["ids"])
    assert_same(t.encode_packed(fx["bytes"], fx["off"]), (fx["ids"], fx["ids_off"]))  # (host path: int32)
    ex.out_bits = 8
    assert L.sw_encode_device_ex(h, d_buf.data_ptr(), len(fx["bytes"]), d_off.data_ptr(), len(fx["off"]) - 1,
                                 ctypes.byref(ex), d_out.data_ptr(), d_oo.data_ptr(), None, None) == _lib.SW_ERR_ARG
    t.close()
    w = sa.Tokenizer(device=0)
    w.merges = {(97, 98): 70000}
    ex.out_bits = 16
    assert L.sw_encode_device_ex(w._encoder(), d_buf.data_ptr(), len(fx["bytes"]), d_off.data_ptr(), len(fx["off"]) - 1,
                                 ctypes.byref(ex), d_out.data_ptr(), d_oo.data_ptr(), None, None) == _lib.SW_ERR_ARG
    w.close()


def test_dedupe_growth_allocation_failure_keeps_table():
    """An allocation failure while growing the dedupe table (forced by SW_OPT_TEST_FAIL_GROWTH) must
    leave the encoder with the table it had: every later launch still equals the oracle, the
    table size is unchanged, and once the failure is lifted growth works again."""
    buf, off = corpus.synth(31, corpus.ENTROPY, 60000, 1074)
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    L, h = _lib.lib(), t._encoder()
    try:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_TEST_FAIL_GROWTH, 1))
        slots0 = None
        for rep in range(3):
            assert_same(gpu_encode(t, buf, off), exp)
            if rep == 0:
                slots0 = L.sw_encoder_get_info(h, _lib.SW_INFO_DEDUPE_SLOTS)
        assert L.sw_encoder_get_info(h, _lib.SW_INFO_DEDUPE_SLOTS) == slots0
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_TEST_FAIL_GROWTH, 0))
        for rep in range(2):
            assert_same(gpu_encode(t, buf, off), exp)
        assert L.sw_encoder_get_info(h, _lib.SW_INFO_DEDUPE_SLOTS) > slots0
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_TEST_FAIL_GROWTH, 0)
        t.close()


def test_shared_handle_patterns_per_call_two_streams():
    """Two tokenizer views with different patterns (cl100k, GPT-2) over ONE device handle
    (Tokenizer.shared), calls interleaved on two streams without host synchronisation between them
    (n_bytes given, sync=False): each result equals the oracle for its own pattern.  The pattern
    travels with the call (sw_encode_ex.pattern), so nothing on the shared handle is raced."""
    import torch
    base = sa.Tokenizer(device=0)
    base.merges = load_model_merges("bl32k.model")
    va, vb = base.shared(""), base.shared(sa.GPT2_PATTERN)
    assert va._encoder().value == vb._encoder().value == base._encoder().value
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    batches = []
    for seed in range(4):
        buf, off = corpus.synth(100 + seed, corpus.MIXED, 2000, 1074)
        batches.append((buf, off, torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev)))
    torch.cuda.synchronize()
    outs = []
    for k, (buf, off, d_buf, d_off) in enumerate(batches):
        for view, st in ((va, s1), (vb, s2)):
            with torch.cuda.stream(st):
                d_out, d_oo = view.encode_device(d_buf, d_off, n_bytes=len(buf), sync=False)
            outs.append((k, view, d_out, d_oo))
    torch.cuda.synchronize()
    for k, view, d_out, d_oo in outs:
        buf, off = batches[k][0], batches[k][1]
        pat = "gpt2" if view is vb else "cl100k"
        exp = oracle_encode(base.merges, buf, off, pat)
        oo = d_oo.cpu().numpy()
        np.testing.assert_array_equal(oo, exp[1])
        np.testing.assert_array_equal(d_out[:int(oo[-1])].cpu().numpy(), exp[0])
    va.close()
    assert base._handle is not None  # (a view never destroys its parent's handle)
    base.close()


@pytest.mark.parametrize("host_presplit", [0, 1])
def test_chunk_dense_tiles_over_the_lds_list(host_presplit):
    """Tiles with more chunk starts than the classification's LDS list holds (1454: runs of
    one-byte strings, "1a1a..." text that cl100k cuts into one-byte chunks, a space between
    letters) go to the overflow kernels (k_split_redo on the device pre-split, k_classify_big on
    a host bitmap) -- the same ids as the oracle, beside ordinary tiles of the same batch."""
    rng = random.Random(5)
    datas = []
    for _ in range(6):
        datas += [bytes([rng.choice(b"abcxyz")]) for _ in range(3000)]      # one-byte strings
        datas.append(("1a" * 2500).encode())                                 # one-byte chunks
        datas.append(" ".join(rng.choice("pqrs") for _ in range(1500)).encode())
        datas.append(b"the quick brown fox jumps over the lazy dog. " * 60)  # ordinary text
    buf, off = pack(datas)
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, host_presplit))
    try:
        assert_same(gpu_encode(t, buf, off), exp)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 0)
