"""The bit-parallel pre-split (csrc/presplit_bits.h: class masks per 32-byte chunk, local window
rules, run carries) run on the CPU chunk by chunk as the device lanes run it
(tests/native/psb_emul.cpp), against the host pre-split (sw_presplit_host, pinned to the
reference's apply_regex through the golden primitives): identical bitmaps for both patterns on
fuzzed Unicode strings, the corpora, long runs that cross many chunks and invalid UTF-8."""
import ctypes
import os
import random
import subprocess
import tempfile

import numpy as np
import pytest

from shredword_amd import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


ALPHABET = ["a", "Z", "s", "l", "ll", "ve", "re", "e", "T", " ", "  ", "\n", "\r\n", "\t", "'", "'s", "'LL", "'ve",
            "'Re", "1", "12345", ".", "!!", "...", "\u00a0", "\u3000", "\u00e9", "\u017f", "\u4e2d\u6587",
            "\U0001f642", "\u0301", "\ud7ff", "x\n\n", " 1", " .", " '", "\x00", "\x7f", "\x0b", "\x85", "\u2028",
            "\u00b2", "\u0663", "word", "Hello", " world"]


def fuzz_strings(seed, n, kmax=40, alphabet=ALPHABET):
    rng = random.Random(seed)
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, kmax))).encode("utf-8", "surrogatepass")
            for _ in range(n)]


@pytest.fixture(scope="module")
def psb():
    d = tempfile.mkdtemp(prefix="psb_emul_")
    so = os.path.join(d, "psb_emul.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "shredword_amd", "csrc"),
                    "-o", so, os.path.join(ROOT, "tests", "native", "psb_emul.cpp")], check=True)
    lib = ctypes.CDLL(so)
    lib.psb_emul.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    lib.psb_emul.restype = ctypes.c_int64

    def run(buf, off, pattern):
        n = int(off[-1] - off[0])
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        buf = np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        slow = lib.psb_emul(buf.ctypes.data, off.ctypes.data, len(off) - 1, pattern, bits.ctypes.data)
        assert slow >= 0, "a second rules() pass still asked for carries"
        return bits, slow
    run.lib = lib
    return run


def check(psb, buf, off, pats=(0, 1, 2)):
    slow = 0
    for pat in pats:
        exp, _ = corpus.presplit(buf, off, pat)
        got, s = psb(buf, off, pat)
        slow += s
        bad = np.nonzero(got != exp[:len(got)])[0]
        if len(bad):
            w = int(bad[0])
            lo = max(0, w * 64 - 16)
            raise AssertionError("pattern %d: first differing word %d (bytes %r)\n got %s\n exp %s" % (
                pat, w, bytes(buf[lo:w * 64 + 80]), bin(int(got[w]))[::-1], bin(int(exp[w]))[::-1]))
    return slow


def test_fuzz_alphabet(psb):
    check(psb, *pack(fuzz_strings(1, 6000)))


def test_fuzz_dense_edges(psb):
    # whitespace / apostrophe / digit heavy: contractions, C runs after O, runs of every kind
    alpha = ["'", "s", "S", "ll", "LL", "ve", "Re", "t", "d", "m", "ſ", " ", "  ", "\n", "\r", "\t", ".", ",", "1",
             "23", "a", "x", "é", "²", "　", "\x85", "😀", "\x0b"]
    check(psb, *pack(fuzz_strings(2, 8000, kmax=60, alphabet=alpha)))


@pytest.mark.parametrize("kind", [corpus.MIXED, corpus.STRESS, corpus.ASCII])
def test_corpora(psb, kind):
    buf, off = corpus.synth(11 + kind, kind, 4000, 700)
    check(psb, buf, off)


def test_long_runs_across_chunks(psb):
    """Runs far longer than the 64-byte window: the carries (digit phase, C runs after an O,
    whitespace runs with a later C) walk over many chunks."""
    datas = [b"1" * 700, b"x" + b"1" * 701 + b"a", b"." + b"\n" * 600 + b" a", b"a" + b"\n" * 300 + b" x",
             b"\n" + b" " * 3000 + b"x", b"\n" + b" " * 3000 + b"\nx", b" " * 3000, b"\t" * 999 + b".",
             b"." + b"\r\n" * 200 + b"\t\tword", "²".encode() * 400 + b"7" * 5, ("٣" * 333).encode(),
             b"x" * 70000, b"'" * 500 + b"s", b"  \n" * 400 + b"y", "　".encode() * 300 + b"\nq",
             "　".encode() * 300 + b"q", b"9" * 95 + b" " + b"8" * 31]
    for shift in range(0, 70, 7):  # the runs at every phase of the chunk grid
        buf, off = pack([b"#" * shift] + datas)
        check(psb, buf, off)


def test_invalid_utf8_and_tiny_strings(psb):
    rng = np.random.default_rng(3)
    datas = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 9)), dtype=np.uint8)) for _ in range(20000)]
    check(psb, *pack(datas))
    rng2 = random.Random(4)
    datas = [bytes(rng2.choice(b"ab \n'\x80\xff\xc3\xa9\xe4\xb8\xf0\x9f\xc5\xbf") for _ in range(rng2.randint(0, 60)))
             for _ in range(4000)]
    check(psb, *pack(datas))


def test_empty_and_single(psb):
    check(psb, *pack([b""]))
    check(psb, *pack([b"a"]))
    check(psb, *pack([b"", b"'", b"s", b"", b"'s", b" ", b"1"]))


def test_fast_class_exhaustive(psb):
    """The pre-split's register fast path for code-point classes (presplit_bits.h fast_class)
    agrees with the UCD tables (exported from `regex`) on every code point it answers."""
    lib = psb.lib
    lib.psb_fast_class_check.argtypes = [ctypes.c_void_p]
    lib.psb_fast_class_check.restype = ctypes.c_int64
    cov = ctypes.c_int64(0)
    assert lib.psb_fast_class_check(ctypes.byref(cov)) == 0
    assert cov.value > 80000  # (CJK, Hangul, CJK extension B, the emoji planes, ...)
