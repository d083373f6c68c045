"""The device pre-split's transducer (csrc/presplit_fsm.h) run on the CPU, segment by segment
exactly as the device lanes split the batch (tests/native/fsm_emul.cpp), against the host
pre-split (sw_presplit_host, pinned to the reference's apply_regex through the golden
primitives): identical bitmaps for every pattern, for 64-byte segments (the kernel's) and
for small odd segment sizes that put a lane boundary at almost every position, so every
resumption rule is exercised.  Both forms are run: the code-point-stepped one (the device's
fallback past its staged window) and the byte-stepped one over per-byte info (its fast path);
and the kernel's own workgroups (presplit_block.h: window, halo, info phase, per-lane parse
with the fallback), thread by thread (mode 2)."""
import ctypes
import os
import random
import subprocess
import tempfile

import numpy as np
import pytest

from shredword_amd import _lib, corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATS = [_lib.SW_PAT_CL100K, _lib.SW_PAT_GPT2, _lib.SW_PAT_NONE]


@pytest.fixture(scope="module")
def emul():
    d = tempfile.mkdtemp(prefix="fsm_emul_")
    so = os.path.join(d, "fsm_emul.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "shredword_amd", "csrc"),
                    "-o", so, os.path.join(ROOT, "tests", "native", "fsm_emul.cpp")], check=True)
    lib = ctypes.CDLL(so)
    lib.fsm_emul.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_int]
    lib.fsm_emul.restype = ctypes.c_int

    def run(buf, off, pattern, seg, byte_stepped):
        n = int(off[-1])
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        buf = np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        lib.fsm_emul(buf.ctypes.data, off.ctypes.data, len(off) - 1, pattern, seg, bits.ctypes.data, byte_stepped)
        return bits
    return run


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


def check(emul, buf, off, segs=(64, 1, 3, 7, 13)):
    for pat in PATS:
        exp, _ = corpus.presplit(buf, off, pat)
        for seg, mode in [(sg, m) for sg in segs for m in (0, 1)] + [(64, 2)]:
            got = emul(buf, off, pat, seg, mode)
            bad = np.nonzero(got != exp[:len(got)])[0]
            if len(bad):
                w = int(bad[0])
                lo = max(0, w * 64 - 16)
                raise AssertionError("pattern %d seg %d mode %d: first differing word %d (bytes %r)\n got %s\n exp %s" % (
                    pat, seg, mode, w, bytes(buf[lo:w * 64 + 80]), bin(int(got[w]))[::-1], bin(int(exp[w]))[::-1]))


ALPHABET = ["a", "Z", "s", "l", "ll", "ve", "re", "e", "T", " ", "  ", "\n", "\r\n", "\t", "'", "'s", "'LL", "'ve",
            "'Re", "1", "12345", ".", "!!", "...", " ", "　", "é", "ſ", "中文",
            "\U0001f642", "́", "퟿", "x\n\n", " 1", " .", " '", "\x00", "\x7f", "\x0b", "\x85", " ",
            "²", "٣", "word", "Hello", " world"]


def fuzz_strings(seed, n, kmax=40, alphabet=ALPHABET):
    rng = random.Random(seed)
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, kmax))).encode("utf-8", "surrogatepass")
            for _ in range(n)]


def test_fuzz_alphabet(emul):
    check(emul, *pack(fuzz_strings(1, 4000)))


def test_fuzz_contractions_and_whitespace(emul):
    small = ["'", "s", "l", "v", "r", "e", "L", "E", "S", "ſ", " ", "\n", "\r", "\t", "!", "1", "a"]
    check(emul, *pack(fuzz_strings(2, 6000, 12, small)))


def test_fuzz_raw_bytes(emul):
    rng = np.random.default_rng(3)
    datas = [bytes(rng.integers(0, 256, size=int(rng.integers(0, 30)), dtype=np.uint8)) for _ in range(3000)]
    # and bytes drawn from the ASCII classes, where the sync rules look
    pool = np.frombuffer(b" \n\r\t'.!-,aZsleT019", dtype=np.uint8)
    datas += [bytes(pool[rng.integers(0, len(pool), size=int(rng.integers(0, 50)))]) for _ in range(3000)]
    check(emul, *pack(datas))


def test_long_runs(emul):
    datas = [b"a" * 5000, b" " * 3000, b"1" * 700, b"!" * 900, b"\n" * 600 + b"a", ("word " * 400).encode(),
             "中".encode() * 300, b"x" * 7000, b"\xff\xfe" * 500, b" \n" * 300 + b" a", b"'" * 200 + b"s",
             b"ab'" * 300, b"12 " * 300, b"\t " * 200 + b"x"]
    check(emul, *pack(datas))


@pytest.mark.parametrize("kind", [corpus.MIXED, corpus.ASCII, corpus.STRESS])
def test_corpora(emul, kind):
    check(emul, *corpus.synth(11, kind, 1500, 700), segs=(64, 5))


def test_device_windows(emul):
    """Parses that run past a workgroup's 2 KiB halo (the fallback over global memory), strings
    crossing many workgroups, and a string that starts exactly where a workgroup's info bytes
    end (byte b0 + 18424: the fallback must settle the string before it)."""
    tail = [b"\n x" * 10000] + fuzz_strings(9, 300)
    for first_len in range(18420, 18429):
        check(emul, *pack([b" " * first_len, b"ab c"] + tail), segs=(64,))
    datas = [b"x" * 70000, "\u4e2d".encode() * 3000, b" " * 5000, b"a" * 2100, ("word " * 4000).encode()]
    check(emul, *pack(datas + tail), segs=(64,))


def test_empty_and_single(emul):
    check(emul, *pack([]))
    check(emul, *pack([b""]))
    check(emul, *pack([b"", b"a", b"", b"", b" ", b""]))
