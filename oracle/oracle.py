"""ORACLE -- TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/libsw_oracle.so (sw_oracle.c).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and only
as the checker (or the timed CPU baseline).  The product (shredword_amd) never imports it.
"""
import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int, c_int32, c_int64, c_uint8, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libsw_oracle.so")
PAT_CL100K, PAT_GPT2, PAT_NONE = 0, 1, 2

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "libsw_oracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_model_new.restype = c_void_p
        L.orc_model_new.argtypes = [POINTER(c_int32), POINTER(c_int32), c_int64]
        L.orc_model_free.argtypes = [c_void_p]
        L.orc_model_get.restype = c_int64
        L.orc_model_get.argtypes = [c_void_p, c_int32, c_int32]
        L.orc_ucd_class.restype = c_int
        L.orc_ucd_class.argtypes = [ctypes.c_uint32]
        L.orc_presplit.restype = c_int64
        L.orc_presplit.argtypes = [POINTER(c_uint8), c_int64, c_int, POINTER(c_int64), c_int64]
        for name in ("orc_encode_chunk", "orc_encode_chunk_naive", "orc_encode_chunk_heap"):
            getattr(L, name).restype = c_int64
            getattr(L, name).argtypes = [c_void_p, POINTER(c_uint8), c_int64, POINTER(c_int32)]
        L.orc_model_well_formed.restype = c_int
        L.orc_model_well_formed.argtypes = [c_void_p]
        L.orc_encode_ordinary.restype = c_int64
        L.orc_encode_ordinary.argtypes = [c_void_p, POINTER(c_uint8), c_int64, c_int, POINTER(c_int32)]
        L.orc_encode_batch.restype = c_int64
        L.orc_encode_batch.argtypes = [c_void_p, POINTER(c_uint8), POINTER(c_int64), c_int64, c_int,
                                       POINTER(c_int32), POINTER(c_int64), c_int]
        L.orc_encode_batch_specials.restype = c_int64
        L.orc_encode_batch_specials.argtypes = [c_void_p, POINTER(c_uint8), POINTER(c_int64), c_int64, c_int,
                                                POINTER(c_uint8), POINTER(c_int64), POINTER(c_int32), c_int64,
                                                POINTER(c_int32), POINTER(c_int64), c_int]
        L.orc_encode_with_specials.restype = c_int64
        L.orc_encode_with_specials.argtypes = [c_void_p, POINTER(c_uint8), c_int64, c_int, POINTER(c_uint8),
                                               POINTER(c_int64), POINTER(c_int32), c_int64, POINTER(c_int32)]
        L.orc_train_words.restype = c_int64
        L.orc_train_words.argtypes = [POINTER(c_uint8), c_int64, c_int32, c_float, POINTER(c_uint8),
                                      POINTER(c_int64), POINTER(c_int64), POINTER(c_uint64), c_int64]
        L.orc_train.restype = c_int64
        L.orc_train.argtypes = [POINTER(c_uint8), c_int64, c_int64, c_int32, c_float, c_uint64,
                                POINTER(c_int32), c_int64, POINTER(c_uint64)]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(POINTER(t))


class OracleModel:
    """merges dict -> oracle hash map."""

    def __init__(self, merges):
        n = len(merges)
        pairs = np.array(list(merges.keys()), dtype=np.int32).reshape(n, 2)
        vals = np.array(list(merges.values()), dtype=np.int32).reshape(n)
        self._h = lib().orc_model_new(_p(pairs, c_int32), _p(vals, c_int32), n)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_model_free(self._h)
            self._h = None

    def get(self, a, b):
        r = lib().orc_model_get(self._h, a, b)
        return None if r < 0 else int(r)

    def encode_chunk(self, data, form=""):
        """form "": the oracle's choice; "naive": the reference loop step by step; "heap": the
        O(n log n) form (well-formed tables only)."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        out = np.empty(max(len(data), 1), dtype=np.int32)
        fn = getattr(lib(), "orc_encode_chunk" + ("_" + form if form else ""))
        n = fn(self._h, _p(buf, c_uint8), len(data), _p(out, c_int32))
        return out[:n].tolist()

    @property
    def well_formed(self):
        return bool(lib().orc_model_well_formed(self._h))

    def encode_ordinary(self, data, pattern=PAT_CL100K):
        if isinstance(data, str):
            data = data.encode("utf-8")
        buf = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        out = np.empty(max(len(data), 1), dtype=np.int32)
        n = lib().orc_encode_ordinary(self._h, _p(buf, c_uint8), len(data), pattern, _p(out, c_int32))
        assert n >= 0
        return out[:n].tolist()

    def encode_batch(self, buf, off, pattern=PAT_CL100K, n_threads=1):
        """-> (ids int32[total], out_off int64[n+1]) for strings buf[off[s]:off[s+1]]."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        n = len(off) - 1
        total = int(off[-1] - off[0]) if n > 0 else 0
        out = np.empty(max(total, 1), dtype=np.int32)
        out_off = np.empty(n + 1, dtype=np.int64)
        if buf.size == 0:
            buf = np.zeros(1, np.uint8)
        t = lib().orc_encode_batch(self._h, _p(buf, c_uint8), _p(off, c_int64), n, pattern, _p(out, c_int32),
                                   _p(out_off, c_int64), n_threads)
        assert t >= 0
        return out[:t], out_off

    def encode_batch_specials(self, buf, off, special_tokens, pattern=PAT_CL100K, n_threads=1):
        """encode_batch with special tokens (dict str -> id, dict order), per string as
        encode_with_specials -> (ids int32[total], out_off int64[n+1])."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        names = [s.encode("utf-8") for s in special_tokens]
        sb = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8)
        so = np.zeros(len(names) + 1, dtype=np.int64)
        np.cumsum([len(x) for x in names], out=so[1:])
        sid = np.array(list(special_tokens.values()) or [0], dtype=np.int32)
        n = len(off) - 1
        total = int(off[-1] - off[0]) if n > 0 else 0
        out = np.empty(max(total, 1), dtype=np.int32)
        out_off = np.empty(n + 1, dtype=np.int64)
        if buf.size == 0:
            buf = np.zeros(1, np.uint8)
        t = lib().orc_encode_batch_specials(self._h, _p(buf, c_uint8), _p(off, c_int64), n, pattern, _p(sb, c_uint8),
                                            _p(so, c_int64), _p(sid, c_int32), len(names), _p(out, c_int32),
                                            _p(out_off, c_int64), n_threads)
        assert t >= 0
        return out[:t], out_off

    def encode_with_specials(self, text, special_tokens, pattern=PAT_CL100K):
        data = text.encode("utf-8")
        names = [s.encode("utf-8") for s in special_tokens]
        sb = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8)
        so = np.zeros(len(names) + 1, dtype=np.int64)
        np.cumsum([len(x) for x in names], out=so[1:])
        sid = np.array(list(special_tokens.values()) or [0], dtype=np.int32)
        buf = np.frombuffer(data or b"\0", dtype=np.uint8)
        out = np.empty(max(len(data), 1), dtype=np.int32)
        n = lib().orc_encode_with_specials(self._h, _p(buf, c_uint8), len(data), pattern, _p(sb, c_uint8),
                                           _p(so, c_int64), _p(sid, c_int32), len(names), _p(out, c_int32))
        assert n >= 0
        return out[:n].tolist()


def presplit(data, pattern=PAT_CL100K):
    """-> list of chunk start byte offsets."""
    if isinstance(data, str):
        data = data.encode("utf-8")
    n = len(data)
    if n == 0:
        return []
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    starts = np.empty(n, dtype=np.int64)
    c = lib().orc_presplit(_p(buf, c_uint8), n, pattern, _p(starts, c_int64), n)
    assert c >= 0
    return starts[:c].tolist()


def ucd_class(cp):
    return lib().orc_ucd_class(cp)


def train(text, target_vocab_size, unk_id=0, character_coverage=0.995, min_pair_freq=2000):
    """The reference BPE trainer restated (sw_train_oracle.c): (merges [m, 3] int32 rows
    (a, b, new_id), final token frequencies [256 + m] uint64)."""
    buf = np.frombuffer(bytes(text), dtype=np.uint8) if not isinstance(text, np.ndarray) else text
    if len(buf) == 0:
        buf = np.zeros(1, np.uint8)[:0]
    cap = max(int(target_vocab_size) - 256, 0)
    rows = np.zeros((max(cap, 1), 3), np.int32)
    freq = np.zeros(256 + max(cap, 1), np.uint64)
    src = buf if len(buf) else np.zeros(1, np.uint8)
    m = lib().orc_train(_p(np.ascontiguousarray(src), c_uint8), len(buf), int(target_vocab_size), int(unk_id),
                        float(character_coverage), int(min_pair_freq), _p(rows, c_int32), cap, _p(freq, c_uint64))
    if m < 0:
        raise ValueError("orc_train failed (%d)" % m)
    return rows[:m].copy(), freq[:256 + m].copy()


def train_words(text, unk_id=0, character_coverage=0.995):
    """Distinct words in the reference's order: (offsets, lengths, counts, kept-char mask)."""
    buf = np.frombuffer(bytes(text), dtype=np.uint8)
    cap = len(buf) // 2 + 16
    off, ln, cnt = np.zeros(cap, np.int64), np.zeros(cap, np.int64), np.zeros(cap, np.uint64)
    keep = np.zeros(256, np.uint8)
    src = buf if len(buf) else np.zeros(1, np.uint8)
    n = lib().orc_train_words(_p(np.ascontiguousarray(src), c_uint8), len(buf), int(unk_id), float(character_coverage),
                              _p(keep, c_uint8), _p(off, c_int64), _p(ln, c_int64), _p(cnt, c_uint64), cap)
    if n < 0:
        raise ValueError("orc_train_words failed (%d)" % n)
    return off[:n].copy(), ln[:n].copy(), cnt[:n].copy(), keep
