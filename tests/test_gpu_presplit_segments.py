"""The device pre-split in segments overlapped with k_classify (SW_OPT_PRESPLIT_SEGMENTS): the
tiles whose bitmap words are not written yet when their segment is classified (the last tile of a
segment, a chunk running past the written words) are deferred to k_classify_deferred.  Every
segment count gives the oracle's ids (oracle/sw_oracle.c), including letter runs of more than a
segment.  All calls go through the C-ABI."""
import numpy as np
import pytest

import oracle
import shredword_amd as sa
from shredword_amd import _lib, corpus
from conftest import PATTERNS, load_model_merges

pytestmark = pytest.mark.gpu
PAT_STR = {"cl100k": "", "gpt2": sa.GPT2_PATTERN}


@pytest.fixture(scope="module", autouse=True)
def need_device():
    if _lib.lib().sw_device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu must run on the MI355X box")


def _batch():
    """~6 MiB: MIXED prose with two 1.4 MiB letter runs (one chunk each under both patterns), one
    starting inside the first segment and one ending the batch."""
    buf, off = corpus.synth(7, corpus.MIXED, 3000, 1074)
    texts = [bytes(buf[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    run = b"ab" * 700_000
    texts.insert(700, b"x " + run + b" y")
    texts.append(b" " + run)
    o = np.zeros(len(texts) + 1, dtype=np.int64)
    np.cumsum([len(s) for s in texts], out=o[1:])
    return np.frombuffer(b"".join(texts), dtype=np.uint8).copy(), o


@pytest.mark.parametrize("pattern", ["cl100k", "gpt2"])
def test_segments_vs_oracle(pattern):
    buf, off = _batch()
    merges = load_model_merges("bl32k.model")
    exp = oracle.OracleModel(merges).encode_batch(buf, off, PATTERNS[pattern], n_threads=8)
    t = sa.Tokenizer(device=0)
    t.merges = merges
    t.pattern = PAT_STR[pattern]
    L = _lib.lib()
    try:
        for segs in (1, 3, 16, 4):
            _lib.check(L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_PRESPLIT_SEGMENTS, segs))
            ids, ids_off = t.encode_packed(buf, off)
            np.testing.assert_array_equal(ids_off, exp[1], err_msg=f"segments={segs}")
            np.testing.assert_array_equal(ids, exp[0], err_msg=f"segments={segs}")
    finally:
        t.close()


def test_segments_option_range():
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges("toy500.model")
    L = _lib.lib()
    try:
        for bad in (0, 17, -1):
            assert L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_PRESPLIT_SEGMENTS, bad) == _lib.SW_ERR_ARG
        assert L.sw_encoder_set_option(t._encoder(), _lib.SW_OPT_PRESPLIT_SEGMENTS, 16) == _lib.SW_OK
    finally:
        t.close()
