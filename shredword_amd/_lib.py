"""ctypes binding of the C-ABI in include/shredword_hip.h and include/shredword_train.h.

Follows the reference's native-binding pattern (`shredword/cbase.py:5-59`): search the package
directory for the built library, `ctypes.CDLL` it, declare argtypes/restype per function, and map
status codes to Python exceptions (as `shredword/trainer.py:14-25` does).  Two deliberate
differences from the reference:
  * the library is loaded lazily, on first use, so `import shredword_amd` never fails on a
    machine without the built library (the reference's `import shredword` raises
    FileNotFoundError at `cbase.py:20`);
  * errors come back as negative status codes plus `sw_last_error()`, never `exit()`.
"""
import ctypes
import os
import sysconfig
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int32, c_int64, c_size_t, c_uint8, c_uint32, c_uint64,
                    c_void_p)

LIB_NAMES = ("libshredword_hip",)

SW_OK = 0
SW_ERR_ARG, SW_ERR_HIP, SW_ERR_ALLOC, SW_ERR_CAP, SW_ERR_NODEV = -1, -2, -3, -4, -5

SW_PAT_CL100K, SW_PAT_GPT2, SW_PAT_NONE = 0, 1, 2
SW_CORPUS_ASCII, SW_CORPUS_MIXED, SW_CORPUS_STRESS, SW_CORPUS_ENTROPY = 0, 1, 2, 3
# options (include/shredword_hip.h)
SW_OPT_PATTERN, SW_OPT_HOST_PRESPLIT, SW_OPT_MAX_LAUNCH_BYTES = 5, 6, 8
SW_OPT_PIPE_RUN_BYTES, SW_OPT_PIPE_DEPTH = 9, 12
SW_OPT_DEVICE_SPECIALS = 18
# measurement and test switches (shredword_amd/csrc/test_options.h; results unchanged)
SW_OPT_CHUNK_TABLE, SW_OPT_DEDUPE, SW_OPT_DEDUPE_SLOTS, SW_OPT_DEDUPE_FP_BITS = 1, 2, 3, 4
SW_OPT_LONG_SPLIT = 7
SW_OPT_DEDUPE_EXACT = 10
SW_OPT_PIPE_COPY_KERNELS = 11
SW_OPT_MERGE_STREAMS = 13
SW_OPT_FUSED_PRESPLIT = 14
SW_OPT_TEST_FAIL_GROWTH = 17
SW_OPT_COMPACT_KERNEL = 19
SW_OPT_STAGED_HEADS = 20
SW_OPT_OUT_BITS = 16  # (removed: set_option rejects it; 16-bit output is sw_encode_ex.out_bits, per call)
SW_INFO_MERGES, SW_INFO_CHUNK_ENTRIES, SW_INFO_WIDE_TABLE, SW_INFO_IDS16, SW_INFO_SPLIT, SW_INFO_DEDUPE_SLOTS = 1, 2, 3, 4, 5, 6
SW_INFO_CHUNK_TABLE_BYTES = 7


class SwStats(Structure):
    _fields_ = [("n_bytes", c_int64), ("n_chunks", c_int64), ("n_tokens", c_int64),
                ("ms_presplit", c_double), ("ms_h2d", c_double), ("ms_kernels", c_double),
                ("ms_d2h", c_double), ("ms_total", c_double)]


class SwSpecials(Structure):
    """sw_specials: the tokenizer's special tokens (UTF-8 bytes, offsets, ids; dict order)."""
    _fields_ = [("bytes", POINTER(c_uint8)), ("off", POINTER(c_int64)), ("ids", POINTER(c_int32)), ("n", c_int64)]


SW_EX_PATTERN = 1


class SwEncodeEx(Structure):
    """sw_encode_ex: per-call choices of sw_encode_device_ex (device pointers as integers).
    pattern: SW_PAT_* for this call (sets SW_EX_PATTERN), or -1 (the default here): the handle's
    SW_OPT_PATTERN.  struct_size is filled in: the library refuses any other layout."""
    _fields_ = [("struct_size", c_int32), ("flags", c_uint32), ("chunk_bits", c_void_p), ("out_bits", c_int32),
                ("sp_pos", c_void_p), ("sp_len", c_void_p), ("sp_id", c_void_p), ("n_sp", c_int64),
                ("pattern", c_int32), ("d_n_sp", c_void_p)]

    def __init__(self, chunk_bits=None, out_bits=32, sp_pos=None, sp_len=None, sp_id=None, n_sp=0, pattern=-1,
                 d_n_sp=None):
        super().__init__(ctypes.sizeof(SwEncodeEx), SW_EX_PATTERN if pattern >= 0 else 0, chunk_bits, out_bits,
                         sp_pos, sp_len, sp_id, n_sp, max(pattern, 0), d_n_sp)


class TrainConfig(Structure):
    """sw_train_config: field for field the reference's BPEConfig (bpe.h:43-48, cbase.py:40)."""
    _fields_ = [("target_vocab_size", c_size_t), ("unk_id", c_int32), ("character_coverage", c_float),
                ("min_pair_freq", c_uint64)]


class ShredwordError(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _get_lib_path():
    """Locate the built library the way cbase.py:_get_lib_path does (package dir, lib/, build/)."""
    override = os.environ.get("SHREDWORD_HIP_LIB")  # e.g. the diagnostic (SW_STAMPS) build
    if override:
        return override
    pkg_dir = os.path.dirname(os.path.abspath(__file__))
    exts = (".so", sysconfig.get_config_var("EXT_SUFFIX") or ".so")
    for d in (pkg_dir, os.path.join(pkg_dir, "lib"), os.path.join(pkg_dir, "..", "build")):
        if not os.path.isdir(d):
            continue
        for f in sorted(os.listdir(d)):
            # variants (libshredword_hip_<name>.so: diagnostics, A/B builds) load only by override
            if f.startswith(LIB_NAMES) and f.endswith(exts) and not f.startswith("libshredword_hip_"):
                return os.path.join(d, f)
    raise FileNotFoundError(
        "libshredword_hip.so not found next to shredword_amd/ -- run "
        "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C shredword_amd`")


_lib = None

# name: (restype, argtypes)
_SIGNATURES = {
    "sw_last_error": (c_char_p, []),
    "sw_version": (c_char_p, []),
    "sw_device_count": (c_int32, []),
    "sw_encoder_create": (c_int32, [POINTER(c_int32), POINTER(c_int32), c_int64, c_int32, POINTER(c_void_p)]),
    "sw_encoder_destroy": (None, [c_void_p]),
    "sw_encoder_reserve": (c_int32, [c_void_p, c_int64, c_int64]),
    "sw_encoder_pin_host": (c_int32, [c_void_p, c_void_p, c_int64]),
    "sw_encoder_unpin_host": (c_int32, [c_void_p, c_void_p]),
    "sw_presplit_host": (c_int64, [POINTER(c_uint8), POINTER(c_int64), c_int64, c_int32, POINTER(c_uint64), c_int32]),
    "sw_encode_batch": (c_int32, [c_void_p, POINTER(c_uint8), POINTER(c_int64), c_int64, c_int32,
                                  POINTER(c_uint64), POINTER(c_int32), c_int64, POINTER(c_int64),
                                  POINTER(SwStats)]),
    "sw_presplit_device": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_void_p,
                                     POINTER(c_int64)]),
    "sw_encode_device": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                   c_void_p, c_void_p, POINTER(c_int64)]),
    "sw_encode_device_ex": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, POINTER(SwEncodeEx), c_void_p,
                                      c_void_p, c_void_p, POINTER(c_int64)]),
    "sw_encode_batch_ex": (c_int32, [c_void_p, POINTER(c_uint8), POINTER(c_int64), c_int64, c_int32,
                                     POINTER(c_uint64), POINTER(SwSpecials), POINTER(c_int32), c_int64,
                                     POINTER(c_int64), POINTER(SwStats)]),
    "sw_find_specials_host": (c_int64, [POINTER(c_uint8), POINTER(c_int64), c_int64, POINTER(SwSpecials),
                                        POINTER(c_int64), POINTER(c_int32), POINTER(c_int32), c_int64, c_int32]),
    "sw_encoder_set_specials": (c_int32, [c_void_p, POINTER(SwSpecials)]),
    "sw_find_specials_device": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                          c_int64, c_void_p, c_void_p, POINTER(c_int64)]),
    "sw_presplit_host_specials": (c_int64, [POINTER(c_uint8), POINTER(c_int64), c_int64, c_int32, POINTER(c_int64),
                                            POINTER(c_int32), c_int64, POINTER(c_uint64), c_int32]),
    "sw_encoder_set_option": (c_int32, [c_void_p, c_int32, c_int64]),
    "sw_encoder_get_info": (c_int64, [c_void_p, c_int32]),
    "sw_encoder_set_timing": (c_int32, [c_void_p, c_int32]),
    "sw_encoder_last_kernel_ms": (c_double, [c_void_p]),
    "sw_encoder_last_classify_ms": (c_double, [c_void_p]),
    "sw_encoder_last_counts": (c_int32, [c_void_p, POINTER(c_int64)]),
    "sw_encoder_phase_cycles": (c_int32, [c_void_p, POINTER(c_double), c_int32]),
    "sw_reassemble_device": (c_int32, [c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int32,
                                       c_void_p, c_void_p, c_void_p]),
    "sw_decoder_create": (c_int32, [POINTER(c_uint8), POINTER(c_int64), POINTER(c_uint8), c_int64, c_int32,
                                    POINTER(c_void_p)]),
    "sw_decoder_destroy": (None, [c_void_p]),
    "sw_decode_batch": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int64), c_int64, POINTER(c_uint8), c_int64,
                                  POINTER(c_int64)]),
    "sw_decode_device": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                   c_void_p, POINTER(c_int64)]),
    "sw_synth_corpus": (c_int64, [c_uint64, c_int32, c_int64, c_int64, POINTER(c_uint8), c_int64,
                                  POINTER(c_int64), c_int32]),
    "sw_synth_splice_specials": (c_int64, [c_uint64, POINTER(c_uint8), POINTER(c_int64), c_int64, POINTER(SwSpecials),
                                           c_double, c_int32, POINTER(c_uint8), c_int64, POINTER(c_int64), c_int32]),
    # trainer (include/shredword_train.h)
    "sw_trainer_create": (c_int32, [POINTER(TrainConfig), c_int32, POINTER(c_void_p)]),
    "sw_trainer_destroy": (None, [c_void_p]),
    "sw_trainer_load_corpus": (c_int32, [c_void_p, c_char_p]),
    "sw_trainer_load_text": (c_int32, [c_void_p, POINTER(c_uint8), c_int64]),
    "sw_trainer_train": (c_int64, [c_void_p]),
    "sw_trainer_merges": (c_int64, [c_void_p, POINTER(c_int32), c_int64]),
    "sw_trainer_token_freq": (c_int64, [c_void_p, POINTER(c_uint64), c_int64]),
    "sw_trainer_save": (c_int32, [c_void_p, c_char_p, c_char_p]),
    "sw_trainer_stats": (c_int32, [c_void_p, POINTER(c_double)]),
}


def lib():
    """Load (once) and return the CDLL with every signature declared."""
    global _lib
    if _lib is None:
        # If PyTorch is present, load it first: it ships its own libamdhip64.so.7 and the
        # process must use ONE HIP runtime (same SONAME => the dynamic linker reuses it).
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        cdll = ctypes.CDLL(_get_lib_path())
        ab = bool(os.environ.get("SHREDWORD_HIP_LIB"))  # (an A/B build of an earlier revision may lack new entry points)
        for name, (res, args) in _SIGNATURES.items():
            if ab and not hasattr(cdll, name):
                continue
            fn = getattr(cdll, name)
            fn.restype = res
            fn.argtypes = args
        _lib = cdll
    return _lib


def exported_symbols():
    return tuple(_SIGNATURES)


def check(code):
    """Map a negative status to ShredwordError (the reference maps -1 to RuntimeError/IOError)."""
    if code < 0:
        msg = lib().sw_last_error()
        raise ShredwordError(int(code), msg.decode("utf-8", "replace") if msg else "")
    return code


def specials_struct(special_tokens):
    """dict str -> id (dict order) -> (SwSpecials, keep-alive arrays)."""
    import numpy as np
    names = [s.encode("utf-8") for s in special_tokens]
    sb = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8).copy()
    so = np.zeros(len(names) + 1, dtype=np.int64)
    np.cumsum([len(x) for x in names], out=so[1:])
    ids = np.array(list(special_tokens.values()) or [0], dtype=np.int64)
    if ids.size and (ids.min() < 0 or ids.max() > 2 ** 31 - 2):
        raise ValueError("special token ids must be in [0, 2^31 - 2]")
    sid = ids.astype(np.int32)
    st = SwSpecials(ptr(sb, c_uint8), ptr(so, c_int64), ptr(sid, c_int32), len(names))
    return st, (sb, so, sid)


def ptr(arr, ctype):
    """ctypes pointer to a contiguous numpy array (None for None)."""
    if arr is None:
        return None
    return arr.ctypes.data_as(POINTER(ctype))
