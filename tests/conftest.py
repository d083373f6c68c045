"""Shared fixtures.  GPU tests carry @pytest.mark.gpu; everything else runs on a CPU-only box."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PATTERNS = {"cl100k": 0, "gpt2": 1, "none": 2}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 device (run with -m gpu on the MI355X box)")


def load_model_merges(name):
    """merges dict of a committed table, parsed like shredword/base.py:135-149."""
    path = os.path.join(GOLD, name)
    if name.endswith(".json"):
        return {(a, b): v for a, b, v in json.load(open(path))}
    m, idx = {}, 256
    with open(path, encoding="utf-8") as f:
        assert f.readline().strip() == "shredword v1"
        f.readline()
        for _ in range(int(f.readline().strip())):
            f.readline()
        for line in f:
            a, b = map(int, line.split())
            m[(a, b)] = idx
            idx += 1
    return m


def golden_index():
    return json.load(open(os.path.join(GOLD, "index.json")))


def load_fixture(entry):
    z = np.load(os.path.join(GOLD, entry["file"]))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def index():
    return golden_index()


@pytest.fixture(scope="session")
def primitives():
    return json.load(open(os.path.join(GOLD, "primitives.json"), encoding="utf-8"))


def page_array(n, dtype, fill=0):
    """A numpy array of n elements on pages of its own (page-aligned start, nothing else on its last
    page), for tests that pin several arrays with Tokenizer.pin_host: two arrays sharing a page
    cannot both be pinned (sw_encoder_pin_host refuses overlapping pages)."""
    import numpy as np
    nbytes = n * np.dtype(dtype).itemsize
    raw = np.empty(nbytes + 2 * 4096, dtype=np.uint8)
    a0 = (-raw.ctypes.data) % 4096
    a = raw[a0:a0 + nbytes].view(dtype)
    a[:] = fill
    return a  # (a view: keeps raw alive)


def page_end_array(n, dtype, fill=0):
    """A numpy array of n elements that ENDS exactly on a page boundary, with at least one page of
    the same allocation after it that nobody pins (so a device access past the array's end would
    touch an unmapped page), and nothing else on its pages.  Its start is wherever n elements put
    it: misaligned to 16 bytes unless n * itemsize is a multiple of 16."""
    import numpy as np
    nbytes = n * np.dtype(dtype).itemsize
    span = (nbytes + 4095) // 4096 * 4096
    raw = np.empty(span + 3 * 4096, dtype=np.uint8)
    base = (-raw.ctypes.data) % 4096  # (first page boundary in raw)
    end = base + span
    a = raw[end - nbytes:end].view(dtype)
    a[:] = fill
    return a
