"""shredword's tokenizer surface (`shredword/base.py`), kept name-for-name so callers can switch.

Primitives and the BaseTokenizer data model with the reference's argument meaning, return
values and error behaviour.  Encode/decode live in `tokenizer.Tokenizer`; the hot path
(pre-split + merge loop) runs natively, never through these Python helpers.
"""
import unicodedata
import warnings
from collections import Counter

import numpy as np

from . import _lib

# Patterns apply_regex may run.  CL100K is the one the reference hard-codes (base.py:56); GPT2 is
# its docstring alternative (base.py:46, in the `(?:...)` spelling) -- the common spelling with
# separate contractions is accepted as the same pattern.
CL100K_PATTERN = r"""'(?i:[sdmt]|ll|ve|re)|[^\r\n\p{L}\p{N}]?+\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]++[\r\n]*|\s*[\r\n]|\s+(?!\S)|\s+"""
GPT2_PATTERN = r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""
GPT2_PATTERN_ALT = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""

_PATTERN_IDS = {"": _lib.SW_PAT_CL100K, CL100K_PATTERN: _lib.SW_PAT_CL100K,
                GPT2_PATTERN: _lib.SW_PAT_GPT2, GPT2_PATTERN_ALT: _lib.SW_PAT_GPT2}

# module-level defaults, as the reference keeps them (base.py:5-8)
merges = {}
vocab = {i: bytes([i]) for i in range(256)}
pattern = ""
special_tokens = {}


_warned_patterns = set()


def pattern_id(pat):
    """Native pre-split id for a tokenizer's `pattern`.

    Policy: "" and the cl100k pattern -> SW_PAT_CL100K, what apply_regex runs
    (base.py:56); the GPT-2 pattern of base.py:46 -> SW_PAT_GPT2; the ints SW_PAT_* as they are.
    Any other pattern string (e.g. the docstring's pattern3/pattern4, base.py:50,54) falls back
    to cl100k with a one-time warning -- the reference's apply_regex ignores the tokenizer's
    pattern and always splits with cl100k, so this keeps its results."""
    if isinstance(pat, (int, np.integer)) and not isinstance(pat, bool):
        if int(pat) not in (_lib.SW_PAT_CL100K, _lib.SW_PAT_GPT2, _lib.SW_PAT_NONE):
            raise ValueError("unknown pre-split id %r (SW_PAT_CL100K, SW_PAT_GPT2 or SW_PAT_NONE)" % (pat,))
        return int(pat)
    if not isinstance(pat, str):
        raise TypeError("pattern must be a str or an SW_PAT_* int, not %s" % type(pat).__name__)
    pid = _PATTERN_IDS.get(pat)
    if pid is None:
        if pat not in _warned_patterns:
            _warned_patterns.add(pat)
            warnings.warn("no native pre-splitter for pattern %r: splitting with the cl100k pattern, as "
                          "shredword's apply_regex does for every tokenizer (base.py:56)" % (pat,),
                          stacklevel=3)
        pid = _lib.SW_PAT_CL100K
    return pid


def get_stats(ids, counts=None):
    """Counts of adjacent pairs of `ids` (base.py:10-20).

    Like the reference, `counts` is accepted but not used: a fresh Counter is returned, keyed in
    first-occurrence order.
    """
    return Counter(zip(ids, ids[1:]))


def merge(ids, pair, idx):
    """Replace each non-overlapping occurrence of `pair`, scanning left to right, by `idx`
    (base.py:22-36).  [1,2,3,1,2],(1,2),4 -> [4,3,4];  [97]*3,(97,97),256 -> [256,97]."""
    out = []
    a, b = pair
    n, i = len(ids), 0
    while i < n:
        if i + 1 < n and ids[i] == a and ids[i + 1] == b:
            out.append(idx)
            i += 2
        else:
            out.append(ids[i])
            i += 1
    return out


def split_chunks(data, pat=""):
    """Chunk byte boundaries of one UTF-8 string under `pat`, computed natively."""
    data = bytes(data)
    n = len(data)
    if n == 0:
        return []
    buf = np.frombuffer(data, dtype=np.uint8)
    off = np.array([0, n], dtype=np.int64)
    bits = np.zeros((n + 63) // 64, dtype=np.uint64)
    L = _lib.lib()
    _lib.check(L.sw_presplit_host(_lib.ptr(buf, _lib.c_uint8), _lib.ptr(off, _lib.c_int64), 1,
                                  pattern_id(pat), _lib.ptr(bits, _lib.c_uint64), 1))
    starts = np.flatnonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:n])
    return starts.tolist()


def apply_regex(text, pat=""):
    """Pre-split `text` into chunks (base.py:38-58), natively.

    The reference always uses the cl100k pattern (base.py:56) whatever `pattern` a tokenizer
    holds; `pat` selects the GPT-2 pattern (base.py:46) or none instead.
    """
    data = text.encode("utf-8")
    starts = split_chunks(data, pat)
    ends = starts[1:] + [len(data)]
    return [data[a:e].decode("utf-8") for a, e in zip(starts, ends)]


def build_vocab(merges, special_tokens):
    """id -> bytes (base.py:60-79): bytes 0..255, then each merge in dict order, then specials."""
    v = {i: bytes([i]) for i in range(256)}
    for (p0, p1), idx in merges.items():
        v[idx] = v[p0] + v[p1]
    for special, idx in special_tokens.items():
        v[idx] = special.encode("utf-8")
    return v


def replace_control_characters(s: str) -> str:
    """Escape category-C characters as \\uXXXX (base.py:81-90)."""
    return "".join(ch if unicodedata.category(ch)[0] != "C" else "\\u%04x" % ord(ch) for ch in s)


def render_token(t: bytes) -> str:
    """Printable form of a token's bytes (base.py:92-96)."""
    return replace_control_characters(t.decode("utf-8", errors="replace"))


class BaseTokenizer:
    """Data model of shredword's BaseTokenizer (base.py:98-149)."""

    def __init__(self):
        self.merges = {}           # (int, int) -> int
        self.pattern = ""
        self.special_tokens = {}   # str -> int
        self.vocab = build_vocab(self.merges, self.special_tokens)

    def train(self, text, vocab_size, verbose=False):
        raise NotImplementedError

    def encode(self, text):
        raise NotImplementedError

    def decode(self, ids):
        raise NotImplementedError

    def save(self, file_prefix):
        """Write `<prefix>.model` ("shredword v1") and the human-readable `<prefix>.vocab`
        (base.py:111-133)."""
        with open(file_prefix + ".model", "w") as f:
            f.write("shredword v1\n")
            f.write(f"{self.pattern}\n")
            f.write(f"{len(self.special_tokens)}\n")
            for special, idx in self.special_tokens.items():
                f.write(f"{special} {idx}\n")
            for a, b in self.merges:
                f.write(f"{a} {b}\n")
        parents = {idx: pair for pair, idx in self.merges.items()}
        with open(file_prefix + ".vocab", "w", encoding="utf-8") as f:
            for idx, token in self.vocab.items():
                s = render_token(token)
                if idx in parents:
                    a, b = parents[idx]
                    f.write(f"[{render_token(self.vocab[a])}][{render_token(self.vocab[b])}] -> [{s}] {idx}\n")
                else:
                    f.write(f"[{s}] {idx}\n")

    def load(self, model_file):
        """Read a "shredword v1" model (base.py:135-149): merge line k gets id 256 + k, and a
        repeated pair keeps its last id."""
        assert model_file.endswith(".model")
        m, specials, nxt = {}, {}, 256
        with open(model_file, "r", encoding="utf-8") as f:
            assert f.readline().strip() == "shredword v1"
            self.pattern = f.readline().strip()
            num_special = int(f.readline().strip())
            for _ in range(num_special):
                tok, tid = f.readline().strip().split()
                specials[tok] = int(tid)
            for line in f:
                a, b = map(int, line.split())
                m[(a, b)] = nxt
                nxt += 1
        self.merges, self.special_tokens = m, specials
        self.vocab = build_vocab(m, specials)

    def load_binary(self, model_file):
        """Read the C++ trainer's binary model: int32 (a, b, new_id) per merge, little endian
        (shredword/csrc/bpe/bpe.cpp:722-731)."""
        raw = np.fromfile(model_file, dtype="<i4")
        if raw.size % 3:
            raise ValueError("%s: size is not a multiple of 12 bytes" % model_file)
        rows = raw.reshape(-1, 3)
        self.merges = {(int(a), int(b)): int(i) for a, b, i in rows}
        self.special_tokens = {}
        self.vocab = build_vocab(self.merges, self.special_tokens)
