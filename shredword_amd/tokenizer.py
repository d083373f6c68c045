"""HIP-backed BPE tokenizer behind shredword's BaseTokenizer surface.

`Tokenizer.encode` is the abstract method of `shredword/base.py:108` made concrete, with the
semantics of the reference's primitives: pre-split with apply_regex (base.py:38-58), bytes to
ids, then repeatedly merge the lowest-ranked adjacent pair (get_stats base.py:10-20, merge
base.py:22-36).  Pre-split runs in native host code, the merge loop in HIP kernels on a gfx950
device.  There is no CPU fallback: without the library or a device, encode raises.
"""
import ctypes
import re

import numpy as np

from . import _lib
from .base import BaseTokenizer, build_vocab, pattern_id


class _TrackedDict(dict):
    """dict that counts its mutations, so the device copy of `merges` is rebuilt when edited."""
    version = 0

    def _bump(self):
        self.version += 1

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self._bump()

    def __delitem__(self, k):
        super().__delitem__(k)
        self._bump()

    def update(self, *a, **k):
        super().update(*a, **k)
        self._bump()

    def clear(self):
        super().clear()
        self._bump()

    def pop(self, *a):
        r = super().pop(*a)
        self._bump()
        return r

    def popitem(self):
        r = super().popitem()
        self._bump()
        return r

    def setdefault(self, k, d=None):
        r = super().setdefault(k, d)
        self._bump()
        return r

    def __ior__(self, other):
        self.update(other)
        return self


def _pack_strings(datas):
    """list of bytes -> (uint8 buffer, int64 offsets[n+1])."""
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    buf = np.frombuffer(b"".join(datas), dtype=np.uint8) if off[-1] else np.zeros(1, np.uint8)
    return buf, off


class Tokenizer(BaseTokenizer):
    """shredword tokenizer whose encode runs on an MI355X.

    Attributes are those of BaseTokenizer (merges, pattern, special_tokens, vocab).  `pattern`
    selects the pre-split (base.pattern_id): "" (default) or the cl100k pattern = what
    apply_regex does; the GPT-2 pattern of base.py:46; any other pattern string falls back to
    cl100k, because the reference's apply_regex ignores the tokenizer's pattern (base.py:56).
    Edits to `merges` (item assignment, update, |=, reassignment) reach the device table on the
    next encode; `vocab` is rebuilt from merges and special_tokens whenever either changed.
    """

    def __init__(self, device=0):
        self._merges = _TrackedDict()
        self._vocab = _TrackedDict()
        self._vocab_key = None
        super().__init__()
        self.device = device
        self._handle = None
        self._handle_key = None
        self._dec = None
        self._dec_key = None
        self._dec_len = None
        self._sp_key = None
        self._sp_re = None
        self.last_stats = None

    # merges is tracked so that edits (README-style `tok.merges[(a, b)] = id`) reach the device
    @property
    def merges(self):
        return self._merges

    @merges.setter
    def merges(self, value):
        d = _TrackedDict(value)
        d.version = self._merges.version + 1
        self._merges = d

    # vocab is tracked too, so in-place edits reach the device decoder
    @property
    def vocab(self):
        return self._vocab

    @vocab.setter
    def vocab(self, value):
        d = _TrackedDict(value)
        d.version = self._vocab.version + 1
        self._vocab = d
        self._vocab_key = self._vocab_source_key()

    def _vocab_source_key(self):
        return (id(self._merges), self._merges.version, tuple(getattr(self, "special_tokens", {}).items()))

    def __del__(self):
        try:
            self.close()
        except (TypeError, AttributeError):  # (interpreter shutdown: module globals already cleared)
            pass

    def close(self):
        h, self._handle = getattr(self, "_handle", None), None
        if h:
            _lib.lib().sw_encoder_destroy(h)
        d, self._dec = getattr(self, "_dec", None), None
        if d:
            _lib.lib().sw_decoder_destroy(d)

    # ---------------------------------------------------------------- training
    def train(self, text, vocab_size, verbose=False, min_pair_freq=2, character_coverage=0.9999, unk_id=-1):
        """Learn `vocab_size - 256` merges from `text` on the GPU (BaseTokenizer.train, abstract in
        the reference, base.py:107; the trainer is shredword's C++ one, bpe.cpp, restated in
        csrc/train.hip: words split at ' \\t\\r\\n', bytes below the character coverage mapped to
        `unk_id`).  The merges replace this tokenizer's (special tokens are kept); merges built on
        a negative `unk_id` are left out (no byte sequence can produce them).  Returns the number
        of merges learned, which is smaller when no pair reaches `min_pair_freq` any more."""
        from .trainer import BPETrainer
        if vocab_size < 256:
            raise ValueError("vocab_size must be at least 256 (the byte alphabet)")
        t = BPETrainer(target_vocab_size=vocab_size, unk_id=unk_id, character_coverage=character_coverage,
                       min_pair_freq=min_pair_freq, device=self.device)
        try:
            t.load_text(text)
            n = t.train()
            rows = t.merges
            freq = t.token_freq if verbose else None
        finally:
            t.destroy()
        made, merges = set(range(256)), {}
        for a, b, v in rows.tolist():
            if a in made and b in made:
                merges[(a, b)] = v
                made.add(v)
        self.merges = merges
        self.vocab = build_vocab(self.merges, self.special_tokens)
        if verbose:
            for k, ((a, b), v) in enumerate(merges.items()):
                print("merge %d/%d: (%d, %d) -> %d (%r) had %d occurrences at the end" % (
                    k + 1, len(merges), a, b, v, self.vocab[v], int(freq[v]) if v < len(freq) else 0))
        return n

    # ---------------------------------------------------------------- device table
    def _encoder(self):
        key = (id(self._merges), self._merges.version, self.device)
        if self._handle is not None and self._handle_key == key:
            return self._handle
        self.close()
        n = len(self._merges)
        pairs = np.array(list(self._merges.keys()), dtype=np.int64).reshape(n, 2)
        vals = np.array(list(self._merges.values()), dtype=np.int64).reshape(n)
        if n and (pairs.min() < 0 or pairs.max() > 0x7FFFFFFF or vals.min() < 0 or vals.max() > 0x7FFFFFFF):
            raise ValueError("merges must map non-negative int32 pairs to values in [0, 2^31-1]")
        pairs = np.ascontiguousarray(pairs, dtype=np.int32)
        vals = np.ascontiguousarray(vals, dtype=np.int32)
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.sw_encoder_create(_lib.ptr(pairs, ctypes.c_int32), _lib.ptr(vals, ctypes.c_int32),
                                       n, int(self.device), ctypes.byref(h)))
        self._handle, self._handle_key = h, key
        return h

    @property
    def ids16(self):
        """True when every id an ordinary encode can produce fits 16 bits (bytes, merge pair
        members and values all < 65536): ids may then travel as 16 bits (shard.reassemble)."""
        key = (id(self._merges), self._merges.version)
        if getattr(self, "_ids16_key", None) != key:
            m = self._merges
            top = max((max(a, b, v) for (a, b), v in m.items()), default=255)
            self._ids16, self._ids16_key = top < 65536, key
        return self._ids16

    # ---------------------------------------------------------------- encode
    def encode_ordinary_batch_np(self, datas):
        """Encode a list of UTF-8 byte strings (no special-token handling) in one device batch.
        Returns (ids int32[total], offsets int64[n+1])."""
        buf, off = _pack_strings(datas)
        return self.encode_packed(buf, off)

    def encode_packed(self, buf, off, chunk_bits=None):
        """Encode the strings buf[off[s]:off[s+1]] (uint8 buffer, int64 offsets) in one device
        batch.  chunk_bits: optional host pre-split bitmap (sw_presplit_host layout).
        Returns (ids int32[total], out_off int64[n+1])."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        if buf.size == 0:
            buf = np.zeros(1, np.uint8)
        n = len(off) - 1
        total = int(off[-1] - off[0]) if n > 0 else 0
        out = np.empty(max(total, 1), dtype=np.int32)
        out_off = np.empty(n + 1, dtype=np.int64)
        stats = _lib.SwStats()
        L = _lib.lib()
        bits = None if chunk_bits is None else np.ascontiguousarray(chunk_bits, dtype=np.uint64)
        _lib.check(L.sw_encode_batch(self._encoder(), _lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64),
                                     n, pattern_id(self.pattern), _lib.ptr(bits, ctypes.c_uint64),
                                     _lib.ptr(out, ctypes.c_int32), total, _lib.ptr(out_off, ctypes.c_int64),
                                     ctypes.byref(stats)))
        self.last_stats = stats
        return out[:int(out_off[-1])], out_off

    def encode_device(self, d_buf, d_off, d_bits=None, d_out=None, d_out_off=None, stream=None):
        """Encode strings already on this tokenizer's device (torch tensors: uint8 bytes, int64
        offsets from 0; optional pre-split bitmap as int64 words, else the device pre-splits with
        `pattern`), on torch's current stream (or `stream`).  Returns (ids int32 [n_tokens],
        offsets int64 [n+1]) as device tensors; the token count is read back (one
        synchronisation).  d_out / d_out_off: optional output buffers (>= n_bytes / n+1)."""
        import torch
        dev = d_buf.device
        n = int(d_off.numel()) - 1
        n_bytes = int(d_off[-1].item()) if n >= 0 else 0
        if d_out is None:
            d_out = torch.empty(max(n_bytes, 1), dtype=torch.int32, device=dev)
        if d_out_off is None:
            d_out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        L = _lib.lib()
        h = self._encoder()
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PATTERN, pattern_id(self.pattern)))
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        n_tok = ctypes.c_int64()
        _lib.check(L.sw_encode_device(h, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n,
                                      d_bits.data_ptr() if d_bits is not None else None,
                                      d_out.data_ptr(), d_out_off.data_ptr(), st, ctypes.byref(n_tok)))
        return d_out[:int(n_tok.value)], d_out_off

    def _split_specials(self, text):
        """Split on special tokens: leftmost occurrence first, dictionary order breaking ties
        (the reference stores special_tokens at base.py:103 but defines no split).  One regex
        alternation of the escaped specials in dict order: `re` takes the leftmost match and,
        at one position, the first alternative that matches -- exactly that rule."""
        key = tuple(self.special_tokens.items())
        if key != self._sp_key:
            specials = [s for s in self.special_tokens if s]
            self._sp_re = re.compile("|".join(map(re.escape, specials))) if specials else None
            self._sp_key = key
        if self._sp_re is None:
            return [text]
        parts, seg = [], 0
        for m in self._sp_re.finditer(text):
            parts.append(text[seg:m.start()])
            parts.append(self.special_tokens[m.group()])
            seg = m.end()
        parts.append(text[seg:])
        return parts

    def encode_batch(self, texts, allowed_special="all"):
        """Encode many strings in one device batch; returns a list of id lists."""
        if allowed_special not in ("all", "none"):
            raise ValueError("allowed_special must be 'all' or 'none'")
        texts = list(texts)
        split = allowed_special == "all" and any(self.special_tokens)
        if not split:  # one piece per text: one device batch, one list conversion
            ids, off = self.encode_ordinary_batch_np([t.encode("utf-8") for t in texts])
            flat, o = ids.tolist(), off.tolist()
            return [flat[o[k]:o[k + 1]] for k in range(len(texts))]
        pieces, layout = [], []
        for t in texts:
            lay = []
            for p in self._split_specials(t):
                if isinstance(p, int):
                    lay.append(p)
                else:
                    lay.append(-1 - len(pieces))
                    pieces.append(p.encode("utf-8"))
            layout.append(lay)
        ids, off = self.encode_ordinary_batch_np(pieces)
        flat, o = ids.tolist(), off.tolist()
        out = []
        for lay in layout:
            r = []
            for x in lay:
                if x >= 0:
                    r.append(x)
                else:
                    r.extend(flat[o[-1 - x]:o[-x]])
            out.append(r)
        return out

    def encode(self, text, allowed_special="all"):
        return self.encode_batch([text], allowed_special)[0]

    def encode_ordinary(self, text):
        return self.encode_batch([text], "none")[0]

    # ---------------------------------------------------------------- decode
    def _vocab_now(self):
        """self.vocab, rebuilt by build_vocab (base.py:60-79) when merges or special_tokens have
        changed since it was last set; a vocab assigned directly is used as it is."""
        if self._vocab_key != self._vocab_source_key():
            self.vocab = build_vocab(self._merges, self.special_tokens)
        return self._vocab

    def _decoder(self):
        """Device copy of the vocabulary (build_vocab, base.py:60-79), rebuilt when it changes."""
        vocab = self._vocab_now()
        key = (id(vocab), vocab.version, self.device)
        if self._dec is not None and self._dec_key == key:
            return self._dec
        d, self._dec = self._dec, None
        if d:
            _lib.lib().sw_decoder_destroy(d)
        n = max(vocab) + 1 if vocab else 0
        lens = np.zeros(n, dtype=np.int64)
        defined = np.zeros(max(n, 1), dtype=np.uint8)
        for i, b in vocab.items():
            lens[i] = len(b)
            defined[i] = 1
        off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        flat = b"".join(vocab[i] for i in sorted(vocab))  # (ascending ids: the offsets' order)
        vb = np.frombuffer(flat or b"\0", dtype=np.uint8)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().sw_decoder_create(_lib.ptr(vb, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64),
                                                _lib.ptr(defined, ctypes.c_uint8), n, int(self.device),
                                                ctypes.byref(h)))
        self._dec, self._dec_key, self._dec_len = h, key, (lens, defined[:n].astype(bool))
        return h

    def decode_packed(self, ids, id_off):
        """Bytes of the id strings ids[id_off[s]:id_off[s+1]] (int32 ids, int64 offsets), decoded on
        the device in one batch.  Returns (uint8 bytes, int64 byte offsets[n+1]).  An id that is
        not in the vocabulary raises KeyError, as vocab[idx] does in the reference."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        id_off = np.ascontiguousarray(id_off, dtype=np.int64)
        h = self._decoder()
        lens, defined = self._dec_len
        sel = ids[int(id_off[0]):int(id_off[-1])] if len(id_off) else ids[:0]
        bad = (sel < 0) | (sel >= len(lens))
        if not bad.any():
            bad = ~defined[sel]
        if bad.any():
            raise KeyError(int(sel[np.flatnonzero(bad)[0]]))
        total = int(lens[sel].sum())
        out = np.empty(max(total, 1), dtype=np.uint8)
        n = len(id_off) - 1
        out_off = np.empty(n + 1, dtype=np.int64)
        _lib.check(_lib.lib().sw_decode_batch(h, _lib.ptr(ids if ids.size else np.zeros(1, np.int32), ctypes.c_int32),
                                              _lib.ptr(id_off, ctypes.c_int64), n, _lib.ptr(out, ctypes.c_uint8),
                                              total, _lib.ptr(out_off, ctypes.c_int64)))
        return out[:total], out_off

    def decode_batch(self, id_lists):
        """Many id lists -> strings (one device batch; UTF-8 errors replaced, per string)."""
        off = np.zeros(len(id_lists) + 1, dtype=np.int64)
        np.cumsum([len(x) for x in id_lists], out=off[1:])
        flat = np.fromiter((i for x in id_lists for i in x), dtype=np.int64, count=int(off[-1]))
        if flat.size and (flat.min() < -2 ** 31 or flat.max() >= 2 ** 31):
            raise KeyError(int(flat[(flat < -2 ** 31) | (flat >= 2 ** 31)][0]))
        buf, boff = self.decode_packed(flat.astype(np.int32), off)
        data = buf.tobytes()
        return [data[boff[k]:boff[k + 1]].decode("utf-8", errors="replace") for k in range(len(id_lists))]

    def decode(self, ids):
        """ids -> str: vocab bytes joined (on the device), undecodable bytes replaced (the
        conventional decode over build_vocab, base.py:60-79)."""
        return self.decode_batch([list(ids)])[0]
