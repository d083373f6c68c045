"""The C-ABI library loads and exports every symbol include/*.h declares.  No compute calls
without a GPU, except the host-only entry points."""
import ctypes
import os
import re

import pytest

from shredword_amd import _lib
from conftest import ROOT


def declared_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(sw_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_symbols_exported():
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.exported_symbols())


def test_version_and_device_count():
    L = _lib.lib()
    assert L.sw_version().startswith(b"shredword_hip")
    assert L.sw_device_count() >= 0


def test_errors_are_status_codes_not_exit():
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.sw_encoder_create(None, None, -1, 0, ctypes.byref(h))
    assert rc == _lib.SW_ERR_ARG
    assert L.sw_last_error()
    assert L.sw_presplit_host(None, None, -1, 0, None, 1) == _lib.SW_ERR_ARG
    assert L.sw_synth_corpus(1, 99, 10, 10, None, 0, None, 1) == _lib.SW_ERR_ARG
    assert L.sw_decoder_create(None, None, None, -1, 0, ctypes.byref(h)) == _lib.SW_ERR_ARG
    assert L.sw_decode_batch(None, None, None, 0, None, 0, None) == _lib.SW_ERR_ARG
    assert L.sw_trainer_create(None, 0, ctypes.byref(h)) == _lib.SW_ERR_ARG
    assert L.sw_trainer_train(None) == _lib.SW_ERR_ARG
    assert L.sw_trainer_save(None, None, None) == _lib.SW_ERR_ARG


def test_no_device_fails_loudly():
    L = _lib.lib()
    if L.sw_device_count() > 0:
        pytest.skip("a device is visible")
    import shredword_amd as sa
    t = sa.Tokenizer()
    t.merges = {(104, 105): 256}
    with pytest.raises(_lib.ShredwordError):
        t.encode("hi")
    with pytest.raises(_lib.ShredwordError):
        sa.BPETrainer(target_vocab_size=300)
