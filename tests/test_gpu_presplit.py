"""Device pre-split (sw_presplit_device) against the host pre-split (sw_presplit_host, itself
pinned to the reference's apply_regex through the `regex` module's outputs in
tests/golden/primitives.json and test_surface.py): the bitmaps must be identical, bit for bit,
for every pattern, on corpora and on the edge cases of the parallel parse (segments with no
sync position, strings crossing workgroups, many tiny strings per workgroup, invalid UTF-8)."""
import ctypes
import random

import numpy as np
import pytest

import shredword_amd as sa
from shredword_amd import _lib, corpus

pytestmark = pytest.mark.gpu

PATS = [_lib.SW_PAT_CL100K, _lib.SW_PAT_GPT2, _lib.SW_PAT_NONE]
_TOK = {}


def _encoder():
    if "t" not in _TOK:
        t = sa.Tokenizer(device=0)
        t.merges = {(104, 105): 256}
        _TOK["t"] = t
    return _TOK["t"]._encoder()


def device_presplit(buf, off, pattern):
    import torch
    dev = torch.device("cuda", 0)
    n = int(off[-1])
    d_buf = torch.from_numpy(np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(dev)
    d_bits = torch.full((max((n + 63) // 64, 1),), -1, dtype=torch.int64, device=dev)  # (must be cleared)
    cnt = ctypes.c_int64()
    # on torch's stream: the fill above is ordered before the library's clear of the bitmap
    _lib.check(_lib.lib().sw_presplit_device(_encoder(), d_buf.data_ptr(), n, d_off.data_ptr(), len(off) - 1, pattern,
                                             d_bits.data_ptr(), torch.cuda.current_stream(dev).cuda_stream,
                                             ctypes.byref(cnt)))
    torch.cuda.synchronize()
    return d_bits.cpu().numpy().view(np.uint64)[:max((n + 63) // 64, 1)], cnt.value


def check(buf, off):
    n = int(off[-1])
    for pat in PATS:
        exp, ecnt = corpus.presplit(buf, off, pat)
        got, gcnt = device_presplit(buf, off, pat)
        if n == 0:
            assert gcnt == 0
            continue
        np.testing.assert_array_equal(got, exp[:len(got)], err_msg="pattern %d" % pat)
        assert gcnt == ecnt


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


@pytest.mark.parametrize("kind,n,mean", [(corpus.MIXED, 20000, 1074), (corpus.ASCII, 20000, 600),
                                         (corpus.STRESS, 20000, 600)])
def test_corpora(kind, n, mean):
    buf, off = corpus.synth(11, kind, n, mean)
    check(buf, off)


def test_edge_strings():
    rng = random.Random(5)
    alphabet = ["a", "Z", " ", "  ", "\n", "\r\n", "\t", "'s", "'LL", "'ve", "1", "12345", ".", "!!", "...", " ",
                "　", "é", "ſ", "中文", "🙂", "́", "퟿", "x\n\n", " 1", " .", "\x00", "\x7f"]
    datas = []
    for _ in range(3000):
        k = rng.randint(0, 40)
        datas.append("".join(rng.choice(alphabet) for _ in range(k)).encode("utf-8", "surrogatepass"))
    datas += [b"", b"", b" ", b"a" * 5000, b" " * 3000, b"1" * 700, b"!" * 900, b"\n" * 600 + b"a",
              ("word " * 4000).encode(), "中" .encode() * 3000, b"x" * 70000, b"\xff\xfe" * 500]
    rng.shuffle(datas)
    buf, off = pack(datas)
    check(buf, off)


def test_invalid_utf8_and_tiny_strings():
    rng = np.random.default_rng(3)
    datas = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 6)), dtype=np.uint8)) for _ in range(60000)]
    buf, off = pack(datas)  # ~150 KB, >512 strings per 16 KiB workgroup: the global-search path
    check(buf, off)


def test_single_huge_string_and_empty():
    check(*pack([b""]))
    check(*pack([]))
    buf, off = corpus.synth(2, corpus.MIXED, 200, 1074)
    check(buf, np.array([0, int(off[-1])], dtype=np.int64))  # one 200 KB string


def test_encode_batch_device_vs_host_presplit():
    """sw_encode_batch pre-splits on the device by default; SW_OPT_HOST_PRESPLIT gives the same ids."""
    t = sa.Tokenizer(device=0)
    from conftest import load_model_merges
    t.merges = load_model_merges("bl32k.model")
    buf, off = corpus.synth(21, corpus.MIXED, 4000, 1074)
    for pat in ("", sa.GPT2_PATTERN):
        t.pattern = pat
        dev_ids = t.encode_packed(buf, off)
        L, h = _lib.lib(), t._encoder()
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 1))
        try:
            host_ids = t.encode_packed(buf, off)
        finally:
            L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 0)
        np.testing.assert_array_equal(dev_ids[0], host_ids[0])
        np.testing.assert_array_equal(dev_ids[1], host_ids[1])


@pytest.mark.parametrize("pattern", PATS)
def test_fused_presplit_runs_across_tiles(pattern):
    """The pre-split fused into the classification (k_split_classify, the default of a device encode
    without a bitmap): runs that cross its 2 KiB tiles -- digit runs of thousands of digits (the
    phase of every third digit), whitespace runs with a \\n far inside or at their end, \\r\\n runs
    after punctuation, a whitespace run ending the batch -- walk past the tile and take
    k_split_redo; the ids must equal those of the host bitmap's encode and of the oracle."""
    import oracle
    rng = random.Random(17 + pattern)
    parts = []
    for k in range(300):
        kind = rng.randrange(6)
        if kind == 0:
            parts.append("".join(rng.choice("0123456789") for _ in range(rng.randint(1500, 6000))))
        elif kind == 1:
            ws = [" "] * rng.randint(100, 4000)
            if rng.random() < 0.7:
                ws[rng.randrange(len(ws))] = "\n"
            parts.append("x" + "".join(ws) + rng.choice(["y", "", "\n", "7"]))
        elif kind == 2:
            parts.append("!!" + "\r\n" * rng.randint(50, 2000) + " z")
        elif kind == 3:
            parts.append("word " * rng.randint(1, 600) + "٣" * rng.randint(1, 3000))
        elif kind == 4:
            parts.append("\t" * rng.randint(1, 3000) + "'s" + "　" * rng.randint(0, 900))
        else:
            parts.append("hello world 123 . " * rng.randint(1, 200))
    datas = [p.encode("utf-8") for p in parts] + [b" " * 5000, b"9" * 4097, b"\n" * 3000]
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    buf = np.frombuffer(b"".join(datas), dtype=np.uint8).copy()
    t = sa.Tokenizer(device=0)
    t.merges = {(48, 49): 256, (32, 32): 257, (257, 257): 258, (10, 10): 259, (119, 111): 260}
    t.pattern = pattern
    fused = t.encode_packed(buf, off)                                  # device pre-split, fused
    host_bits, _ = corpus.presplit(buf, off, pattern)
    hosted = t.encode_packed(buf, off, host_bits)                      # host bitmap, k_classify
    np.testing.assert_array_equal(fused[1], hosted[1])
    np.testing.assert_array_equal(fused[0], hosted[0])
    exp = oracle.OracleModel(t.merges).encode_batch(buf, off, pattern, n_threads=8)
    np.testing.assert_array_equal(fused[0], exp[0])
    np.testing.assert_array_equal(fused[1], exp[1])
    t.close()
