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


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirrors of the C-ABI structs have the header's sizes and field offsets (a C
    program compiled against include/shredword_hip.h prints them), and the option / info numbers
    in _lib.py are the headers' (public ones in include/, test switches in csrc/test_options.h)."""
    import subprocess
    structs = {"sw_encode_ex": _lib.SwEncodeEx, "sw_stats": _lib.SwStats, "sw_specials": _lib.SwSpecials}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "shredword_hip.h"', '#include "test_options.h"',
           'int main(void) {']
    for cname, py in structs.items():
        src.append('  printf("%s size %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            src.append('  printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    consts = [n for n in dir(_lib) if re.match(r"SW_(OPT|INFO|PAT|EX)_", n) and n != "SW_OPT_OUT_BITS"]
    for n in consts:
        src.append('  printf("%s %%d\\n", (int)(%s));' % (n, n))
    src.append("  return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-I",
                    os.path.join(ROOT, "shredword_amd", "csrc"), "-o", str(exe), str(c)], check=True)
    got = dict(ln.rsplit(" ", 1) for ln in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got["%s size" % cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got["%s.%s" % (cname, f)]) == getattr(py, f).offset, (cname, f)
    for n in consts:
        assert int(got[n]) == getattr(_lib, n), n
    ex = _lib.SwEncodeEx(pattern=1)
    assert ex.struct_size == ctypes.sizeof(_lib.SwEncodeEx) and ex.flags == _lib.SW_EX_PATTERN and ex.pattern == 1
    assert _lib.SwEncodeEx().flags == 0  # (the handle's pattern)
