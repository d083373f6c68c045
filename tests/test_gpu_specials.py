"""Special tokens (E1) through the native path: the occurrences found on the host threads, each one
chunk encoding to its id on the GPU, the text between them pre-split on its own -- on the device
(k_split_classify with the occurrences' ends as string boundaries) or on the host
(sw_presplit_host_specials) -- against the oracle's orc_encode_with_specials (pinned: the pieces are
ordinary encodes, pinned to the reference's primitives by the golden vectors).

The reference stores special_tokens (shredword/base.py:103) but defines no split; the rule is the
build's (leftmost first, dict order on ties), the one tests/test_specials.py pins on the host."""
import ctypes
import os
import random

import numpy as np
import pytest

import oracle
import shredword_amd as sa
from shredword_amd import _lib, corpus
from conftest import GOLD, load_model_merges

pytestmark = pytest.mark.gpu

SPECIALS = {"<|endoftext|>": 100257, "<|fim_prefix|>": 100258, "<|fim|>": 100259, "<|": 100260}
PAT = {"cl100k": oracle.PAT_CL100K, "gpt2": oracle.PAT_GPT2, "none": oracle.PAT_NONE}


def tok_for(model, pattern="cl100k"):
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges(model)
    t.pattern = {"cl100k": "", "gpt2": sa.GPT2_PATTERN, "none": _lib.SW_PAT_NONE}[pattern]
    return t


def expected(t, buf, off, specials, pattern):
    return oracle.OracleModel(t.merges).encode_batch_specials(buf, off, specials, PAT[pattern], n_threads=8)


def fuzz_texts(seed, n, kmax=60):
    rng = random.Random(seed)
    alphabet = ["word", " the", " ", "  ", "\n", "\n\n", "123", "45678", "'s", "'LL", "!!", "...", " <", "|", ">",
                "<|fim|>", "<|endoftext|>", "<|fim_prefix|>", "<|", "中文", "\U0001f642", "été", "\t", "\r\n",
                " x", "aaaa", "Hello", " world"]
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, kmax))) for _ in range(n)]


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


@pytest.mark.parametrize("pattern", ["cl100k", "gpt2", "none"])
@pytest.mark.parametrize("host_presplit", [0, 1])
def test_encode_batch_specials_fuzz(pattern, host_presplit):
    """Tokenizer.encode_batch with special tokens (the native path) == the oracle, device and host
    pre-split, on fuzzed strings full of specials, partial specials, empty strings."""
    t = tok_for("bl32k.model", pattern)
    t.special_tokens = dict(SPECIALS)
    texts = fuzz_texts(3 + host_presplit, 1500) + ["", "<|endoftext|>", "<|endoftext|><|endoftext|>", "<|fim", "x<|"]
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, host_presplit))
    try:
        got = t.encode_batch(texts)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 0)
    om = oracle.OracleModel(t.merges)
    for i, s in enumerate(texts):
        assert got[i] == om.encode_with_specials(s, SPECIALS, PAT[pattern]), (i, s)
    # allowed_special="none": the specials' text is ordinary text
    assert t.encode_batch(texts[:50], "none") == [om.encode_with_specials(s, {}, PAT[pattern]) for s in texts[:50]]
    t.close()


def test_golden_gpt2_fixture_with_specials():
    """The enc_bl32k_gpt2 golden strings: as they are, the native path gives the reference-generated
    ids; with specials spliced in, the oracle's."""
    fx = np.load(os.path.join(GOLD, "enc_bl32k_gpt2.npz"))
    t = tok_for("bl32k.model", "gpt2")
    t.special_tokens = dict(SPECIALS)
    ids, off = t.encode_packed(fx["bytes"], fx["off"], specials=SPECIALS)
    np.testing.assert_array_equal(ids, fx["ids"])
    np.testing.assert_array_equal(off, fx["ids_off"])
    buf, soff = corpus.splice_specials(fx["bytes"], fx["off"], SPECIALS, per_kib=8.0, end_special=0)
    ids, off = t.encode_packed(buf, soff, specials=SPECIALS)
    e_ids, e_off = expected(t, buf, soff, SPECIALS, "gpt2")
    np.testing.assert_array_equal(off, e_off)
    np.testing.assert_array_equal(ids, e_ids)
    t.close()


def test_device_entry_specials_and_bitmap():
    """sw_encode_device_ex with device occurrences: the fused device pre-split (no bitmap) and a host
    bitmap from sw_presplit_host_specials give the oracle's ids; 16-bit output with specials is
    refused."""
    import torch
    t = tok_for("bl50k.model")
    texts = [s.encode() for s in fuzz_texts(9, 3000, 120)]
    buf, off = pack(texts)
    pos, ln, ids = corpus.find_specials(buf, off, SPECIALS)
    assert len(pos) > 1000
    e_ids, e_off = expected(t, buf, off, SPECIALS, "cl100k")
    dev = torch.device("cuda", 0)
    d_buf, d_off = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev)
    d_sp = tuple(torch.from_numpy(x).to(dev) for x in (pos, ln, ids))
    g_ids, g_off = t.encode_device(d_buf, d_off, d_specials=d_sp)
    np.testing.assert_array_equal(g_off.cpu().numpy(), e_off)
    np.testing.assert_array_equal(g_ids.cpu().numpy(), e_ids)
    bits, _ = corpus.presplit_specials(buf, off, pos, ln, _lib.SW_PAT_CL100K)
    d_bits = torch.from_numpy(bits.view(np.int64)).to(dev)
    g_ids, g_off = t.encode_device(d_buf, d_off, d_bits=d_bits, d_specials=d_sp)
    np.testing.assert_array_equal(g_ids.cpu().numpy(), e_ids)
    with pytest.raises(_lib.ShredwordError):
        t.encode_device(d_buf, d_off, d_specials=d_sp, out_bits=16)
    t.close()


def test_specials_tile_edges_and_long_occurrences():
    """Occurrences across the 2 KiB tile and 32-byte lane edges, a special longer than a tile, runs of
    adjacent occurrences, strings that are only specials."""
    long_sp = "<|" + "x" * 3000 + "|>"
    sp = {"<|endoftext|>": 100257, long_sp: 100261, "<|fim|>": 100259}
    t = tok_for("bl32k.model")
    t.special_tokens = sp
    rng = random.Random(5)
    texts = []
    for k in range(200):
        pre = "a" * rng.randint(0, 2100) + " word 12345"
        texts.append(pre + rng.choice(list(sp)) * rng.randint(1, 4) + " tail" * rng.randint(0, 30))
    texts += [long_sp, long_sp + long_sp, "<|fim|>" * 500, "<|endoftext|> " * 300]
    got = t.encode_batch(texts)
    om = oracle.OracleModel(t.merges)
    for i, s in enumerate(texts):
        assert got[i] == om.encode_with_specials(s, sp, oracle.PAT_CL100K), i
    t.close()


def test_pipelined_batch_with_specials():
    """A host batch above the pipeline's run size (runs of whole strings, each run's occurrences
    rebased) and above the launch limit (SW_OPT_MAX_LAUNCH_BYTES), with ids over 16 bits (32-bit
    downloads) -- equal to the oracle."""
    t = tok_for("bl32k.model", "gpt2")
    t.special_tokens = dict(SPECIALS)
    buf, off = corpus.synth(21, corpus.MIXED, 6000, 900, n_threads=8)
    buf, off = corpus.splice_specials(buf, off, SPECIALS, per_kib=1.5, end_special=0)
    e_ids, e_off = expected(t, buf, off, SPECIALS, "gpt2")
    L, h = _lib.lib(), t._encoder()
    try:
        for opt, val in ((_lib.SW_OPT_PIPE_RUN_BYTES, 1 << 20), (_lib.SW_OPT_MAX_LAUNCH_BYTES, 1 << 20)):
            _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, val if opt == _lib.SW_OPT_PIPE_RUN_BYTES else 0))
            _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, val if opt == _lib.SW_OPT_MAX_LAUNCH_BYTES else 0))
            out = np.zeros(len(buf), dtype=np.int32)
            g_ids, g_off = t.encode_packed(buf, off, specials=SPECIALS, out=out)
            np.testing.assert_array_equal(g_off, e_off)
            np.testing.assert_array_equal(g_ids, e_ids)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 128 << 20)
        L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, 0)
    t.close()


def _device_find(t, buf, off):
    import torch
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(buf if len(buf) else np.zeros(1, np.uint8)).to(dev)
    d_off = torch.from_numpy(off - off[0]).to(dev)
    pos, ln, ids, cnt, n = t.find_specials_device(d_buf, d_off, n_bytes=int(off[-1] - off[0]), sync=True)
    assert int(cnt.item()) == n
    return pos[:n].cpu().numpy(), ln[:n].cpu().numpy(), ids[:n].cpu().numpy()


@pytest.mark.parametrize("case", range(9))
def test_device_finder_equals_host_finder(case):
    """sw_find_specials_device == sw_find_specials_host (itself == the plain restatement split_ref,
    tests/test_specials.py) on adversarial sets: specials that overlap themselves and each other
    ("aa", "aaa", "ab"/"ba" chains, "<|a" inside "<|a|>"), more than four distinct first bytes (the
    LDS bit-set path), an empty special, occurrences across 32-byte lanes and 2 KiB tiles, strings
    cut inside a special, long runs of one letter (clusters of overlapping candidates)."""
    rng = random.Random(100 + case)
    sets = [
        {"aa": 300, "aaa": 301},
        {"aaa": 301, "aa": 300, "a": 299},
        {"ab": 310, "ba": 311, "aba": 312},
        {"<|a|>": 320, "<|a": 321, "|>": 322, "": 323},
        {"x": 330, "yz": 331, "<|endoftext|>": 332, "\n\n": 333, "é": 334, "\U0001f642": 335, "q" * 64: 336},
        dict(SPECIALS),
        {"the": 340, " the": 341, "he": 342, "e ": 343},
        {"\n": 350, "\n\n": 351, " ": 352},
        # one first byte, shared prefixes past the 16 bytes k_sp_find's records hold, dict order
        # putting a longer special before its prefix and after it
        {"<|im_start|>assistant": 360, "<|im_start|>": 361, "<|im_start|>assistant_long": 362,
         "<|im_start|>user": 363, "<|im_end|>": 364, "<|im_start|>assistan": 365},
    ]
    sp = sets[case]
    t = tok_for("bl32k.model")
    t.special_tokens = sp
    names = [k for k in sp if k] + ["a", "b", "|", "<", ">", " ", "\n", "word", "é", "th", "e", "assistant", "_long"]
    datas = []
    for k in range(400):
        n_parts = rng.choice([0, 1, 5, 40, 300, 1200])
        datas.append("".join(rng.choice(names) for _ in range(n_parts)).encode("utf-8"))
    datas += [b"a" * 5000, b"ab" * 3000, b"<|a|>" * 900, b"", b"aa", b"a"]
    buf, off = pack(datas)
    h_pos, h_len, h_id = corpus.find_specials(buf, off, sp)
    d_pos, d_len, d_id = _device_find(t, buf, off)
    np.testing.assert_array_equal(d_pos, h_pos)
    np.testing.assert_array_equal(d_len, h_len)
    np.testing.assert_array_equal(d_id, h_id)
    # a sub-batch starting at an odd byte: positions relative to its first byte
    sub = off[3:200]
    h2 = corpus.find_specials(buf, sub, sp)
    d2 = _device_find(t, buf[int(sub[0]):int(sub[-1])].copy(), sub)
    for a, b in zip(d2, h2):
        np.testing.assert_array_equal(a, b)
    t.close()


@pytest.mark.parametrize("order", [0, 1])
def test_long_self_overlapping_run(order):
    """A cluster far longer than k_sp_find's window (a 4 MiB run of one letter with "aa" and "aaa",
    both dict orders) goes to the global path, whose walk takes 32 positions a step from a window
    staged in LDS: equal to the host finder, and bounded in time (the walk of one candidate a
    step of table loads took ~1 us a position)."""
    import time
    import torch
    sp = {"aa": 300, "aaa": 301} if order == 0 else {"aaa": 301, "aa": 300}
    t = tok_for("bl32k.model")
    t.special_tokens = sp
    buf, off = pack([b"x" + b"a" * (4 << 20) + b"y", b"ab" * 100, b"a" * 7, b"aaaa" * 3000])
    d_buf = torch.from_numpy(buf).to("cuda:0")
    d_off = torch.from_numpy(off).to("cuda:0")
    t0 = time.perf_counter()
    pos, ln, ids, cnt, n = t.find_specials_device(d_buf, d_off, sync=True)
    dt = time.perf_counter() - t0
    h_pos, h_len, h_id = corpus.find_specials(buf, off, sp)
    np.testing.assert_array_equal(pos[:n].cpu().numpy(), h_pos)
    np.testing.assert_array_equal(ln[:n].cpu().numpy(), h_len)
    np.testing.assert_array_equal(ids[:n].cpu().numpy(), h_id)
    assert dt < 1.5, dt
    t.close()


@pytest.mark.parametrize("pattern", ["cl100k", "gpt2"])
def test_encode_with_device_found_specials(pattern):
    """The whole specials path on the device: find (sw_find_specials_device) -> encode
    (sw_encode_device_ex with the count left on the device) with no synchronisation between them;
    and sw_encode_batch_ex with the device finder (SW_OPT_DEVICE_SPECIALS 1, the default) and the
    host threads' finder (0), pipelined and not -- all equal to the oracle."""
    import torch
    t = tok_for("bl32k.model", pattern)
    t.special_tokens = dict(SPECIALS)
    texts = [s.encode() for s in fuzz_texts(31, 4000, 150)]
    buf, off = pack(texts)
    e_ids, e_off = expected(t, buf, off, SPECIALS, pattern)
    dev = torch.device("cuda", 0)
    d_buf, d_off = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev)
    found = t.find_specials_device(d_buf, d_off, n_bytes=len(buf))
    g_ids, g_off = t.encode_device(d_buf, d_off, d_specials=found, n_bytes=len(buf))
    np.testing.assert_array_equal(g_off.cpu().numpy(), e_off)
    np.testing.assert_array_equal(g_ids.cpu().numpy(), e_ids)
    L, h = _lib.lib(), t._encoder()
    try:
        for dev_sp in (1, 0):
            _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEVICE_SPECIALS, dev_sp))
            for run in (0, 1 << 16):  # (one launch; the pipeline's runs)
                _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, run))
                ids, o = t.encode_packed(buf, off, specials=SPECIALS)
                np.testing.assert_array_equal(o, e_off)
                np.testing.assert_array_equal(ids, e_ids)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_DEVICE_SPECIALS, 1)
        L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 128 << 20)
    t.close()


@pytest.mark.parametrize("per_kib", [64, 300])
def test_dense_specials_device_path(per_kib):
    """Special-dense batches (64 and 300 occurrences per KiB, the bench's `dense` corpus and
    denser): more occurrences in a tile's index range than one wave's 64 probes, so the window's
    first-occurrence search (sp_first_end_wave) takes its multi-step path; the device finder and
    the encode against the oracle, GPT-2 and cl100k."""
    import torch
    bench_sp = {"<|endoftext|>": 50256, "<|fim_prefix|>": 50257, "<|fim_middle|>": 50258, "<|fim_suffix|>": 50259}
    buf0, off0 = corpus.synth(5, corpus.MIXED, 3000, 1074)
    buf, off = corpus.splice_specials(buf0, off0, bench_sp, per_kib=per_kib, end_special=0)
    dev = torch.device("cuda", 0)
    d_buf, d_off = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev)
    for pattern in ("gpt2", "cl100k"):
        t = tok_for("bl32k.model", pattern)
        t.special_tokens = dict(bench_sp)
        e_ids, e_off = expected(t, buf, off, bench_sp, pattern)
        found = t.find_specials_device(d_buf, d_off, n_bytes=len(buf))
        g_ids, g_off = t.encode_device(d_buf, d_off, d_specials=found, n_bytes=len(buf))
        np.testing.assert_array_equal(g_off.cpu().numpy(), e_off)
        np.testing.assert_array_equal(g_ids.cpu().numpy(), e_ids)
        t.close()


def test_short_special_budget_fallback_and_ex_struct_checks():
    """A one-byte special: its worst case (an occurrence at every byte) on a 40 MB batch is over the
    device finder's memory budget, so sw_encode_batch_ex finds the occurrences on the host threads;
    on a small batch the device finds them -- the oracle's ids either way.  sw_encode_device_ex
    refuses a struct of another size and an unknown per-call pattern."""
    import torch
    sp = {"\n": 100300, "<|endoftext|>": 100257}
    t = tok_for("bl32k.model")
    t.special_tokens = sp
    for n_str, mean in ((200, 300), (60000, 700)):
        buf, off = corpus.synth(33, corpus.MIXED, n_str, mean, n_threads=8)
        ids, got_off = t.encode_packed(buf, off, specials=sp)
        e_ids, e_off = expected(t, buf, off, sp, "cl100k")
        np.testing.assert_array_equal(got_off, e_off)
        np.testing.assert_array_equal(ids, e_ids)
    L, h = _lib.lib(), t._encoder()
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(buf[:4096].copy()).to(dev)
    d_off = torch.tensor([0, 4096], dtype=torch.int64, device=dev)
    d_out = torch.empty(4096, dtype=torch.int32, device=dev)
    d_oo = torch.empty(2, dtype=torch.int64, device=dev)
    for bad in ("size", "pattern"):
        ex = _lib.SwEncodeEx()
        if bad == "size":
            ex.struct_size = 0
        else:
            ex.flags, ex.pattern = _lib.SW_EX_PATTERN, 7
        rc = L.sw_encode_device_ex(h, d_buf.data_ptr(), 4096, d_off.data_ptr(), 1, ctypes.byref(ex), d_out.data_ptr(),
                                   d_oo.data_ptr(), None, None)
        assert rc == _lib.SW_ERR_ARG, bad
    t.close()
