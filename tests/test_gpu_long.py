"""Long chunks on the GPU (long_split.h: split + verify over the whole GPU, well-formed tables)
against the oracle: letter runs of 64 KiB .. 1 MiB (one cl100k chunk each), strings of the same
sizes encoded with pattern "none" (one chunk of mixed text each), (a, a) and whitespace runs,
many long chunks in one batch, and the wave loop (SW_OPT_LONG_SPLIT 0) on moderate sizes.
The oracle's long-chunk form (orc_encode_chunk_heap) is checked against the reference loop in
tests/test_oracle_golden.py.  Reference loop: shredword/base.py:10-36."""
import random
import time

import numpy as np
import pytest

import oracle
import shredword_amd as sa
from shredword_amd import _lib, corpus
from conftest import PATTERNS, load_model_merges

pytestmark = pytest.mark.gpu

_TOKS = {}


def tok_for(model, mode=1):
    """A tokenizer of `model` whose long chunks take SW_OPT_LONG_SPLIT `mode` (1: split + verify
    over the whole GPU; 0: the wave loop per chunk)."""
    if (model, mode) not in _TOKS:
        t = sa.Tokenizer(device=0)
        t.merges = load_model_merges(model)
        _lib.check(_lib.lib().sw_encoder_set_option(t._encoder(), _lib.SW_OPT_LONG_SPLIT, mode))
        _TOKS[model, mode] = t
    return _TOKS[model, mode]


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


def check(t, datas, pattern):
    buf, off = pack(datas)
    t.pattern = {"cl100k": "", "gpt2": sa.GPT2_PATTERN, "none": 2}[pattern]
    got = t.encode_packed(buf, off)
    exp = oracle.OracleModel(t.merges).encode_batch(buf, off, PATTERNS[pattern], n_threads=8)
    np.testing.assert_array_equal(got[1], exp[1])
    np.testing.assert_array_equal(got[0], exp[0])
    return got


def letters(rng, n):
    return bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(n))


@pytest.mark.parametrize("model", ["bl50k.model", "bl32k.model"])
@pytest.mark.parametrize("size", [65536, 262144, 1 << 20])
def test_letter_run(model, size):
    t = tok_for(model)
    assert _lib.lib().sw_encoder_get_info(t._encoder(), _lib.SW_INFO_SPLIT) == 1
    rng = random.Random(size)
    data = np.frombuffer(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(4096)), np.uint8)
    run = np.resize(data, size)  # (a 4 KiB random pattern repeated: one letter chunk of `size` bytes)
    run[::4099] = np.frombuffer(letters(rng, len(run[::4099])), np.uint8)
    check(t, [b"x", run.tobytes(), b" y"], "cl100k")
    # one launch, timed (the encode of a 1 MiB chunk takes milliseconds, not seconds)
    buf, off = pack([run.tobytes()])
    t.encode_packed(buf, off)
    t0 = time.perf_counter()
    t.encode_packed(buf, off)
    dt = time.perf_counter() - t0
    print("%s %d-byte letter run: %.2f ms (host call, kernels %.2f ms)" % (model, size, dt * 1e3,
                                                                         t.last_stats.ms_kernels))
    assert t.last_stats.ms_kernels < 200.0


@pytest.mark.parametrize("size", [65536, 1 << 20])
def test_pattern_none_long_strings(size):
    """Pattern "none": a whole string is one chunk (mixed UTF-8 prose of 64 KiB / 1 MiB)."""
    t = tok_for("bl32k.model")
    buf, off = corpus.synth(77, corpus.MIXED, size // 1000 + 8, 1074)
    text = buf.tobytes()[:size]
    cut = len(text)
    while cut > 0 and (text[cut - 1] & 0xC0) == 0x80:  # (whole code points)
        cut -= 1
    check(t, [text[:cut - 1], b"tail", text[:5000]], "none")
    t.pattern = ""


@pytest.mark.parametrize("mode", [1, 0])
def test_runs_and_whitespace(mode):
    """(a, a) runs and whitespace runs cascade junction conflicts: windows grow over rounds."""
    t = tok_for("bl50k.model", mode)
    datas = [b"a" * 100000, b"ab" * 30000, b" " * 50000 + b"x", b"\n" * 3000 + b" z", b"zz" + b"e" * 5001,
             b"aaab" * 2500, b"  " + b"\t" * 777 + b"q", b"ll" * 999 + b"lll"]
    check(t, datas, "cl100k")
    check(t, [d[:4000] for d in datas], "none")


@pytest.mark.parametrize("mode", [1, 0])
def test_many_long_chunks_one_batch(mode):
    """Thousands of long chunks of every length in one launch with short ones between them."""
    t = tok_for("bl50k.model", mode)
    rng = random.Random(9)
    datas = []
    for i in range(3000):
        n = rng.choice([33, 34, 40, 47, 64, 65, 100, 511, 512, 513, 1000, 4095, 4096, 4097, 9000])
        datas.append(letters(rng, n))
        datas.append(b" the " + bytes(rng.choice(b"0123456789") for _ in range(rng.randint(1, 9))))
    check(t, datas, "cl100k")
    t.pattern = ""


@pytest.mark.parametrize("size", [2000, 16384])
def test_wave_loop_option(size):
    """SW_OPT_LONG_SPLIT 0: every long chunk runs the exact wave loop (the ill-formed tables'
    path) -- the same ids."""
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges("bl50k.model")
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_LONG_SPLIT, 0))
    rng = random.Random(size)
    check(t, [letters(rng, size), b"a" * size, letters(rng, 77)], "cl100k")
    t.close()
