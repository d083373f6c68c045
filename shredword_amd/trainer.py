"""BPETrainer: the reference's trainer surface (shredword/trainer.py:5-39) over the MI355X trainer
(include/shredword_train.h): the pair histogram and every merge's corpus rewrite run on the GPU,
the heap on the host; the merges are the reference trainer's (tests/golden/train_*).

    t = BPETrainer(target_vocab_size=8192, unk_id=0, character_coverage=0.995, min_pair_freq=2000)
    t.load_corpus("corpus.txt")
    t.train()
    t.save("out.model", "out.vocab")      # binary int32 triples + "token freq" lines (bpe.cpp:678-739)
    tok = t.tokenizer()                   # the merges as an encode-ready Tokenizer

No CPU fallback: without a GPU the constructor raises ShredwordError (SW_ERR_NODEV).
"""
import ctypes

import numpy as np

from . import _lib


class BPETrainer:
    def __init__(self, target_vocab_size=8192, unk_id=0, character_coverage=0.995, min_pair_freq=2000, device=0):
        self.config = _lib.TrainConfig(target_vocab_size=target_vocab_size, unk_id=unk_id,
                                       character_coverage=character_coverage, min_pair_freq=min_pair_freq)
        self.trainer = None
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().sw_trainer_create(ctypes.byref(self.config), int(device), ctypes.byref(h)))
        self.trainer = h

    def load_corpus(self, path: str):
        """bpe_load_corpus (bpe.cpp:208-297); IOError as the reference's wrapper raises.

        One difference: a corpus holding NUL bytes is rejected (IOError).  The reference reads it
        with fgets + strtok (bpe.cpp:230-251), which silently drops the rest of a line after a
        NUL, up to its 4096-byte read buffer's boundary -- behaviour that depends on that buffer's
        size, so it is not restated."""
        if _lib.lib().sw_trainer_load_corpus(self.trainer, path.encode("utf-8")) != 0:
            raise IOError(f"Failed to load corpus from {path}: {_lib.lib().sw_last_error().decode()}")

    def load_text(self, text):
        """The same from memory (str is UTF-8 encoded)."""
        data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
        _lib.check(_lib.lib().sw_trainer_load_text(self.trainer, _lib.ptr(buf, ctypes.c_uint8), len(data)))

    def train(self):
        """bpe_train (bpe.cpp:597-655); returns the number of merges performed."""
        n = _lib.lib().sw_trainer_train(self.trainer)
        if n < 0:
            raise RuntimeError(f"Training failed: {_lib.lib().sw_last_error().decode()}")
        return int(n)

    @property
    def merges(self):
        """[m, 3] int32 rows (left, right, new id)."""
        L = _lib.lib()
        n = _lib.check(L.sw_trainer_merges(self.trainer, None, 0))
        rows = np.zeros((max(n, 1), 3), dtype=np.int32)
        _lib.check(L.sw_trainer_merges(self.trainer, _lib.ptr(rows, ctypes.c_int32), n))
        return rows[:n]

    @property
    def token_freq(self):
        L = _lib.lib()
        n = _lib.check(L.sw_trainer_token_freq(self.trainer, None, 0))
        freq = np.zeros(max(n, 1), dtype=np.uint64)
        _lib.check(L.sw_trainer_token_freq(self.trainer, _lib.ptr(freq, ctypes.c_uint64), n))
        return freq[:n]

    @property
    def stats(self):
        """ms: load, upload, histogram + heap seed, waiting on the device rewrites, host work on
        the critical path (pops, launches, change application not hidden behind a merge launched
        ahead); then merges, distinct words, symbols."""
        out = (ctypes.c_double * 8)()
        _lib.check(_lib.lib().sw_trainer_stats(self.trainer, out))
        keys = ("ms_load", "ms_upload", "ms_histogram", "ms_rewrites", "ms_host_apply", "merges", "words", "symbols")
        return dict(zip(keys, list(out)))

    def save(self, model_path: str, vocab_path: str):
        _lib.check(_lib.lib().sw_trainer_save(self.trainer, model_path.encode("utf-8"), vocab_path.encode("utf-8")))

    def tokenizer(self, device=0):
        """The trained merges as a Tokenizer (merge value = new id, as the .model format).  Merges
        with a negative member (the UNK id when unk_id < 0), and transitively the merges built on
        them, are left out: no byte sequence can produce them, so the encodings are the same (and
        build_vocab, base.py:60-79, can render every kept merge)."""
        from .tokenizer import Tokenizer
        tok = Tokenizer(device)
        made, merges = set(range(256)), {}
        for a, b, v in self.merges.tolist():
            if a in made and b in made:
                merges[(a, b)] = v
                made.add(v)
        tok.merges = merges
        return tok

    def destroy(self):
        if self.trainer:
            _lib.lib().sw_trainer_destroy(self.trainer)
            self.trainer = None

    def __del__(self):
        try:
            self.destroy()
        except (TypeError, AttributeError):  # (interpreter shutdown: module globals already cleared)
            pass
