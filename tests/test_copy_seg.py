"""The pipeline's copy kernels' addressing (csrc/copy_seg.h) on the CPU: tests/native/copy_seg_emul.cpp
runs the device template itself, lane by lane, with the realigning shuffle emulated for whole
waves, and checks every access for every source / destination misalignment and every length class
(n mod 16, heads longer than n, several blocks per lane): writes exactly [dst, dst + n), each byte
once with the source's value; reads only 16-byte aligned blocks that hold a byte of the source
range (so never a page outside it).  The round-4 copy (unaligned 16-byte accesses, encode.hip before
commit 0685c92) is checked the same way under the stricter rule that every read lies inside
[src, src + n) -- DESIGN.md §4.5 uses both results."""
import ctypes
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LENGTHS = list(range(0, 49)) + [63, 64, 65, 255, 256, 257, 1023, 1024, 1025] + list(range(2040, 2057))


@pytest.fixture(scope="module")
def emul():
    d = tempfile.mkdtemp(prefix="copy_seg_emul_")
    so = os.path.join(d, "copy_seg_emul.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "shredword_amd", "csrc"),
                    "-o", so, os.path.join(ROOT, "tests", "native", "copy_seg_emul.cpp")], check=True)
    lib = ctypes.CDLL(so)
    lib.copy_seg_check.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                   ctypes.c_char_p, ctypes.c_int]
    lib.copy_seg_check.restype = ctypes.c_int
    return lib


def run_all(lib, version, nts):
    msg = ctypes.create_string_buffer(256)
    bad = []
    for nt in nts:
        for n in LENGTHS:
            for sm in range(16):
                for dm in range(16):
                    if lib.copy_seg_check(version, n, sm, dm, nt, msg, len(msg)):
                        bad.append(msg.value.decode())
    return bad


@pytest.mark.parametrize("nt", [64, 128])
def test_copy_seg_ranges_every_alignment(emul, nt):
    """The current copy (aligned destination stores, aligned source blocks realigned by a shuffle)."""
    bad = run_all(emul, 0, [nt])
    assert not bad, bad[:5]


def test_round4_copy_ranges_every_alignment(emul):
    """The round-4 copy that ran when the pinned-output fault was seen: every access inside its range."""
    bad = run_all(emul, 1, [64, 128])
    assert not bad, bad[:5]
