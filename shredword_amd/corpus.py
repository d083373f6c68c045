"""Synthetic corpora for the benchmark configs, generated natively.

Deterministic for a given (seed, kind, n_strings, mean_len) on any machine and thread count.
"""
import ctypes

import numpy as np

from . import _lib

ASCII, MIXED, STRESS, ENTROPY = _lib.SW_CORPUS_ASCII, _lib.SW_CORPUS_MIXED, _lib.SW_CORPUS_STRESS, _lib.SW_CORPUS_ENTROPY


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


def splice_specials(buf, off, special_tokens, per_kib=1.0, end_special=0, seed=7, n_threads=0):
    """The corpus (buf, off) with special tokens (dict str -> id) inserted: about per_kib random ones
    per KiB of each string at code-point boundaries, and the end_special-th one at every string's
    end (None: none) -> (bytes, offsets)."""
    L = _lib.lib()
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    st, keep = _lib.specials_struct(special_tokens)
    n = len(off) - 1
    out_off = np.empty(n + 1, dtype=np.int64)
    es = -1 if end_special is None else int(end_special)
    total = _lib.check(L.sw_synth_splice_specials(seed, _lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64),
                                                  n, ctypes.byref(st), float(per_kib), es, None, 0,
                                                  _lib.ptr(out_off, ctypes.c_int64), n_threads))
    out = np.empty(max(total, 1), dtype=np.uint8)
    _lib.check(L.sw_synth_splice_specials(seed, _lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64), n,
                                          ctypes.byref(st), float(per_kib), es, _lib.ptr(out, ctypes.c_uint8), total,
                                          _lib.ptr(out_off, ctypes.c_int64), n_threads))
    del keep
    return out[:total], out_off


def find_specials(buf, off, special_tokens, n_threads=0):
    """Special-token occurrences (sw_find_specials_host): (pos int64, len int32, id int32) arrays,
    positions relative to off[0]."""
    L = _lib.lib()
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    st, keep = _lib.specials_struct(special_tokens)
    n = len(off) - 1
    cnt = _lib.check(L.sw_find_specials_host(_lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64), n,
                                             ctypes.byref(st), None, None, None, 0, n_threads))
    pos = np.empty(max(cnt, 1), dtype=np.int64)
    ln = np.empty(max(cnt, 1), dtype=np.int32)
    ids = np.empty(max(cnt, 1), dtype=np.int32)
    if cnt:
        _lib.check(L.sw_find_specials_host(_lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64), n,
                                           ctypes.byref(st), _lib.ptr(pos, ctypes.c_int64), _lib.ptr(ln, ctypes.c_int32),
                                           _lib.ptr(ids, ctypes.c_int32), cnt, n_threads))
    del keep
    return pos[:cnt], ln[:cnt], ids[:cnt]


def presplit_specials(buf, off, sp_pos, sp_len, pattern=_lib.SW_PAT_CL100K, n_threads=0):
    """Host pre-split bitmap with special-token occurrences (sw_presplit_host_specials) and the chunk count."""
    L = _lib.lib()
    n = int(off[-1] - off[0]) if len(off) else 0
    bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
    sp_pos = np.ascontiguousarray(sp_pos, dtype=np.int64)
    sp_len = np.ascontiguousarray(sp_len, dtype=np.int32)
    cnt = _lib.check(L.sw_presplit_host_specials(_lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64),
                                                 len(off) - 1, pattern, _lib.ptr(sp_pos, ctypes.c_int64),
                                                 _lib.ptr(sp_len, ctypes.c_int32), len(sp_pos),
                                                 _lib.ptr(bits, ctypes.c_uint64), n_threads))
    return bits, cnt
