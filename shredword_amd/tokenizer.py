"""HIP-backed BPE tokenizer behind shredword's BaseTokenizer surface.

`Tokenizer.encode` is the abstract method of `shredword/base.py:108` made concrete, with the
semantics of the reference's primitives: pre-split with apply_regex (base.py:38-58), bytes to
ids, then repeatedly merge the lowest-ranked adjacent pair (get_stats base.py:10-20, merge
base.py:22-36).  Pre-split runs in native host code, the merge loop in HIP kernels on a gfx950
device.  There is no CPU fallback: without the library or a device, encode raises.
"""
import ctypes

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
        self.last_stats = None
        self._parent = None  # (a view made by shared(): encodes through the parent's device table)

    def shared(self, pattern=None):
        """A tokenizer that uses this one's merges and its device handle (one copy of the tables on
        the device) with its own `pattern` and special tokens: several such views may encode
        concurrently, on different streams, each with its own pattern (the pattern is passed per
        call, never set on the shared handle).  The view does not own the handle."""
        v = Tokenizer(self.device)
        v._parent = self
        v._merges = self._merges
        v.special_tokens = dict(self.special_tokens)
        v.pattern = self.pattern if pattern is None else pattern
        return v

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
        if h and getattr(self, "_parent", None) is None:
            _lib.lib().sw_encoder_destroy(h)  # (unpins whatever pin_host pinned)
        self._pinned = []
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
        if self._parent is not None:
            if self._merges is not self._parent._merges:
                raise RuntimeError("a shared() view's merges must stay its parent's")
            return self._parent._encoder()
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

    def encode_packed(self, buf, off, chunk_bits=None, specials=None, out=None, out_off=None):
        """Encode the strings buf[off[s]:off[s+1]] (uint8 buffer, int64 offsets) in one device
        batch.  chunk_bits: optional host pre-split bitmap (sw_presplit_host layout; with specials,
        sw_presplit_host_specials').  specials: None (ordinary encode) or a dict str -> id of special
        tokens to split on (sw_encode_batch_ex: found by the library's host threads, no Python loop).
        out / out_off: optional caller arrays (int32 [>= total bytes], int64 [n+1], e.g. reused or
        pinned across calls, so the ids are not written into a freshly page-faulted array).
        Returns (ids int32[n_tokens] -- a view of out when given --, out_off int64[n+1])."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        if buf.size == 0:
            buf = np.zeros(1, np.uint8)
        n = len(off) - 1
        total = int(off[-1] - off[0]) if n > 0 else 0
        if out is None:
            out = np.empty(max(total, 1), dtype=np.int32)
        elif out.dtype != np.int32 or not out.flags["C_CONTIGUOUS"] or out.size < total:
            raise ValueError("out: a contiguous int32 array of at least the batch's byte count")
        if out_off is None:
            out_off = np.empty(n + 1, dtype=np.int64)
        elif out_off.dtype != np.int64 or not out_off.flags["C_CONTIGUOUS"] or out_off.size < n + 1:
            raise ValueError("out_off: a contiguous int64 array of at least n + 1 entries")
        stats = _lib.SwStats()
        L = _lib.lib()
        bits = None if chunk_bits is None else np.ascontiguousarray(chunk_bits, dtype=np.uint64)
        args = (self._encoder(), _lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64), n,
                pattern_id(self.pattern), _lib.ptr(bits, ctypes.c_uint64))
        tail = (_lib.ptr(out, ctypes.c_int32), max(out.size, total), _lib.ptr(out_off, ctypes.c_int64), ctypes.byref(stats))
        if specials:
            st, keep = _lib.specials_struct(specials)
            _lib.check(L.sw_encode_batch_ex(*args, ctypes.byref(st), *tail))
            del keep
        else:
            _lib.check(L.sw_encode_batch(*args, *tail))
        self.last_stats = stats
        return out[:int(out_off[n])], out_off[:n + 1]

    def pin_host(self, arr):
        """Pin a host numpy array this tokenizer's encode_packed will read (the bytes) or write
        (out= / out_off=) call after call: its pages are locked and mapped for the device, so the
        input is read over PCIe without a staging copy and the ids / offsets are written by the
        device into the caller's arrays (sw_encoder_pin_host).  Keep the array alive until
        unpin_host(arr) or close()."""
        if not arr.flags["C_CONTIGUOUS"] or arr.nbytes == 0:
            raise ValueError("pin_host: a non-empty contiguous array")
        _lib.check(_lib.lib().sw_encoder_pin_host(self._encoder(), arr.ctypes.data, arr.nbytes))
        self._pinned = getattr(self, "_pinned", [])
        self._pinned.append(arr)  # (kept alive while pinned)

    def unpin_host(self, arr):
        _lib.check(_lib.lib().sw_encoder_unpin_host(self._encoder(), arr.ctypes.data))
        self._pinned = [a for a in getattr(self, "_pinned", []) if a.ctypes.data != arr.ctypes.data]

    def encode_device(self, d_buf, d_off, d_bits=None, d_out=None, d_out_off=None, stream=None, out_bits=32,
                      d_specials=None, n_bytes=None, sync=True):
        """Encode strings already on this tokenizer's device (torch tensors: uint8 bytes, int64
        offsets from 0; optional pre-split bitmap as int64 words, else the device pre-splits with
        `pattern`), on torch's current stream (or `stream`).  out_bits 16: the ids are written as
        16 bits (int16 tensor holding each id's low 16 bits; tables whose every id fits, the
        multi-GPU transport).  d_specials: optional special-token occurrences on the device,
        (pos int64, len int32, id int32) as corpus.find_specials gives them (a caller bitmap must
        then come from presplit_specials).  d_out / d_out_off: optional output buffers (>= n_bytes
        of the output dtype / n+1).

        The pattern goes with the call (sw_encode_ex.pattern), so tokenizers with different patterns
        may share one handle and call from several streams.  n_bytes: the batch's byte count
        (d_off[-1]); None reads it back from the device (one synchronisation).  sync=True returns
        (ids [n_tokens], offsets int64 [n+1]), the token count read back (one synchronisation);
        sync=False enqueues the work and returns (d_out, d_out_off) whole, without waiting: the
        count is d_out_off[-1] on the device."""
        import torch
        if out_bits not in (16, 32):
            raise ValueError("out_bits must be 16 or 32")
        dev = d_buf.device
        n = int(d_off.numel()) - 1
        if n_bytes is None:
            n_bytes = int(d_off[-1].item()) if n >= 0 else 0
        n_bytes = int(n_bytes)
        if n_bytes > d_buf.numel():
            raise ValueError("n_bytes exceeds d_buf")
        want = torch.int16 if out_bits == 16 else torch.int32
        if d_out is None:
            d_out = torch.empty(max(n_bytes, 1), dtype=want, device=dev)
        elif d_out.dtype != want or d_out.numel() < n_bytes:
            raise ValueError("d_out: %s with at least n_bytes elements" % want)
        if d_out_off is None:
            d_out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        L = _lib.lib()
        h = self._encoder()
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        ex = _lib.SwEncodeEx(d_bits.data_ptr() if d_bits is not None else None, out_bits,
                             pattern=pattern_id(self.pattern))
        if d_specials is not None and d_specials[0].numel() > 0:
            pos, ln, ids = d_specials[:3]
            if pos.dtype != torch.int64 or ln.dtype != torch.int32 or ids.dtype != torch.int32:
                raise ValueError("d_specials: (int64 positions, int32 lengths, int32 ids[, int64 device count])")
            ex.sp_pos, ex.sp_len, ex.sp_id, ex.n_sp = pos.data_ptr(), ln.data_ptr(), ids.data_ptr(), pos.numel()
            if len(d_specials) > 3:  # (find_specials_device's: the count stays on the device)
                ex.d_n_sp = d_specials[3].data_ptr()
        n_tok = ctypes.c_int64()
        _lib.check(L.sw_encode_device_ex(h, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n, ctypes.byref(ex),
                                         d_out.data_ptr(), d_out_off.data_ptr(), st,
                                         ctypes.byref(n_tok) if sync else None))
        if not sync:
            return d_out, d_out_off
        return d_out[:int(n_tok.value)], d_out_off

    def find_specials_device(self, d_buf, d_off, n_bytes=None, stream=None, sync=False):
        """The occurrences of self.special_tokens in strings already on the device (as encode_device
        takes them), found on the device (sw_find_specials_device: leftmost first, dict order at one
        position -- sw_find_specials_host's rule, bit for bit).  Returns (pos int64, len int32, id int32,
        count int64[1]) device tensors sized for the worst case; the first `count` entries are the
        occurrences.  Pass the tuple as encode_device(d_specials=...): the count is read on the
        device, nothing synchronises.  sync=True also returns the count as an int (one
        synchronisation).  Specials longer than 64 bytes need the host finder (ValueError)."""
        import torch
        L = _lib.lib()
        h = self._encoder()
        specials = {k: v for k, v in self.special_tokens.items()}
        st, keep = _lib.specials_struct(specials)
        _lib.check(L.sw_encoder_set_specials(h, ctypes.byref(st)))
        del keep
        dev = d_buf.device
        n = int(d_off.numel()) - 1
        if n_bytes is None:
            n_bytes = int(d_off[-1].item()) if n >= 0 else 0
        lens = [len(k.encode("utf-8")) for k in specials if k]
        if lens and max(lens) > 64:
            raise ValueError("a special token over 64 bytes: use the host finder (corpus.find_specials)")
        cap = int(n_bytes) // max(min(lens), 1) + 1 if lens else 1
        pos = torch.empty(cap, dtype=torch.int64, device=dev)
        ln = torch.empty(cap, dtype=torch.int32, device=dev)
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        stream_h = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        n_host = ctypes.c_int64()
        _lib.check(L.sw_find_specials_device(h, d_buf.data_ptr(), int(n_bytes), d_off.data_ptr(), n, pos.data_ptr(),
                                             ln.data_ptr(), ids.data_ptr(), cap, cnt.data_ptr(), stream_h,
                                             ctypes.byref(n_host) if sync else None))
        if sync:
            return pos, ln, ids, cnt, int(n_host.value)
        return pos, ln, ids, cnt

    def encode_batch(self, texts, allowed_special="all"):
        """Encode many strings in one device batch; returns a list of id lists.  allowed_special
        "all": occurrences of self.special_tokens encode to their ids -- leftmost first, the first
        special in dict order at one position (the reference stores special_tokens, base.py:103,
        but defines no split) -- found by the library's host threads; "none": ordinary text."""
        if allowed_special not in ("all", "none"):
            raise ValueError("allowed_special must be 'all' or 'none'")
        texts = list(texts)
        specials = self.special_tokens if allowed_special == "all" and any(self.special_tokens) else None
        ids, off = self.encode_packed(*_pack_strings([t.encode("utf-8") for t in texts]), specials=specials)
        flat, o = ids.tolist(), off.tolist()
        return [flat[o[k]:o[k + 1]] for k in range(len(texts))]

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
