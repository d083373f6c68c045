"""Synthetic corpora for the benchmark configs, generated natively.

Deterministic for a given (seed, kind, n_strings, mean_len) on any machine and thread count.
"""
import ctypes

import numpy as np

from . import _lib

ASCII, MIXED, STRESS = _lib.SW_CORPUS_ASCII, _lib.SW_CORPUS_MIXED, _lib.SW_CORPUS_STRESS


def synth(seed, kind, n_strings, mean_len, n_threads=0):
    """-> (bytes uint8[total], offsets int64[n_strings+1])."""
    L = _lib.lib()
    off = np.empty(n_strings + 1, dtype=np.int64)
    total = _lib.check(L.sw_synth_corpus(seed, kind, n_strings, mean_len, None, 0,
                                         _lib.ptr(off, ctypes.c_int64), n_threads))
    buf = np.empty(max(total, 1), dtype=np.uint8)
    _lib.check(L.sw_synth_corpus(seed, kind, n_strings, mean_len, _lib.ptr(buf, ctypes.c_uint8), total,
                                 _lib.ptr(off, ctypes.c_int64), n_threads))
    return buf[:total], off


def presplit(buf, off, pattern=_lib.SW_PAT_CL100K, n_threads=0):
    """Host pre-split bitmap (uint64 words, bit i = byte i starts a chunk) and the chunk count."""
    L = _lib.lib()
    n = int(off[-1] - off[0]) if len(off) else 0
    bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
    cnt = _lib.check(L.sw_presplit_host(_lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64),
                                        len(off) - 1, pattern, _lib.ptr(bits, ctypes.c_uint64), n_threads))
    return bits, cnt
