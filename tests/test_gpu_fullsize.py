"""Full-size parity at the bench's own configurations (BASELINE.json configs[1], [2], [4]): the
exact batches bench.py times, encoded by the HIP path and compared id for id with the oracle
(oracle/sw_oracle.c on the box's host threads), which is itself pinned to the reference's
primitives at scale by tests/test_oracle_golden.py (digests of >= 16 MB per corpus made with
shredword/base.py, oracle/make_golden.py).  Reference loop: base.py:10-58.

  C2  1 GiB MIXED, 1M strings, 32k merges, cl100k pre-split on the GPU   (bench.py default)
  C5  631 MB STRESS, 1M strings, 50k merges, cl100k pre-split on the GPU (bench.py --config c5)
  C3  64 MB of the C2 corpus with special tokens spliced in, GPT-2 pre-split + specials on the
      host, GPU merge loop; and the bench's own C3-with-specials batch (bench.py --specials 1:
      the C2 corpus with specials spliced in, cut to one launch), device and host pre-split
  ENTROPY  the low-repetition corpus (bench.py --corpus entropy), 1 GiB, 32k merges"""
import ctypes
import os
import random

import numpy as np
import pytest

import oracle
import shredword_amd as sa
from shredword_amd import _lib, corpus
from conftest import load_model_merges

pytestmark = pytest.mark.gpu

THREADS = min(16, len(os.sched_getaffinity(0)))
BENCH_SEED = 1_000_003  # bench.py: corpus.synth(1_000_003 + rank, ...)


def device_encode(tok, buf, off, reps=1):
    """The bench's step: sw_encode_device on HBM-resident torch buffers, device pre-split; reps
    launches on the same encoder (the dedupe table is cleared by the launches themselves, and grows
    after one that overflowed it): every launch's (ids, offsets)."""
    import torch
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.empty(len(buf), dtype=torch.int32, device=dev)
    d_oo = torch.empty(len(off), dtype=torch.int64, device=dev)
    n_tok = ctypes.c_int64()
    outs = []
    for _ in range(reps):
        d_out.fill_(-7)
        _lib.check(_lib.lib().sw_encode_device(tok._encoder(), d_buf.data_ptr(), len(buf), d_off.data_ptr(),
                                               len(off) - 1, None, d_out.data_ptr(), d_oo.data_ptr(),
                                               torch.cuda.current_stream(dev).cuda_stream, ctypes.byref(n_tok)))
        outs.append((d_out[:n_tok.value].cpu().numpy(), d_oo.cpu().numpy()))
    del d_buf, d_off, d_out, d_oo
    torch.cuda.empty_cache()
    return outs if reps > 1 else outs[0]


def first_mismatch(got, exp):
    n = min(len(got), len(exp))
    bad = np.nonzero(got[:n] != exp[:n])[0]
    return int(bad[0]) if len(bad) else n


@pytest.mark.parametrize("cfg", ["c2", "c5", "entropy"])
def test_bench_batch_vs_oracle(cfg):
    kind, mean, model = {"c2": (corpus.MIXED, 1074, "bl32k.model"), "c5": (corpus.STRESS, 600, "bl50k.model"),
                         "entropy": (corpus.ENTROPY, 1074, "bl32k.model")}[cfg]
    buf, off = corpus.synth(BENCH_SEED, kind, 1_000_000, mean, n_threads=THREADS)
    if cfg == "c2":
        assert len(buf) == 1_073_322_961  # (the bench's C2 batch, BENCH_r02)
    tok = sa.Tokenizer(device=0)
    tok.merges = load_model_merges(model)
    # ENTROPY overflows the first launch's dedupe table (~15 M distinct chunks): the second launch
    # grows it, the third runs on the grown table -- every launch against the oracle
    reps = 3 if cfg == "entropy" else 1
    outs = device_encode(tok, buf, off, reps)
    outs = outs if reps > 1 else [outs]
    exp_ids, exp_off = oracle.OracleModel(tok.merges).encode_batch(buf, off, oracle.PAT_CL100K, n_threads=THREADS)
    for got_ids, got_off in outs:
        assert len(got_ids) == len(exp_ids), (len(got_ids), len(exp_ids), first_mismatch(got_ids, exp_ids))
        assert np.array_equal(got_off, exp_off)
        i = first_mismatch(got_ids, exp_ids)
        assert i == len(exp_ids), "first differing id at %d" % i
    if cfg == "entropy":
        assert _lib.lib().sw_encoder_get_info(tok._encoder(), _lib.SW_INFO_DEDUPE_SLOTS) > (1 << 22)
    tok.close()


def test_c3_specials_gpt2_64mb_vs_oracle():
    """C3: 64 MB of the C2 corpus as text with special tokens spliced in; the specials split and
    the GPT-2 pre-split on the host (SW_OPT_HOST_PRESPLIT), the merge loop on the GPU."""
    buf, off = corpus.synth(BENCH_SEED, corpus.MIXED, 62_000, 1074, n_threads=THREADS)
    specials = {"<|endoftext|>": 100257, "<|fim_prefix|>": 100258, "<|fim|>": 100259}
    rng = random.Random(12)
    names = list(specials)
    texts = []
    for s in range(len(off) - 1):
        t = bytes(buf[off[s]:off[s + 1]]).decode("utf-8")
        for _ in range(rng.randint(0, 3)):  # specials at random code-point positions
            k = rng.randint(0, len(t))
            t = t[:k] + rng.choice(names) + t[k:]
        texts.append(t)
    assert sum(len(t.encode()) for t in texts) > 64_000_000
    tok = sa.Tokenizer(device=0)
    tok.merges = load_model_merges("bl32k.model")
    tok.pattern = sa.GPT2_PATTERN
    tok.special_tokens = specials
    om = oracle.OracleModel(tok.merges)
    exp = [om.encode_with_specials(t, specials, oracle.PAT_GPT2) for t in texts]
    L, h = _lib.lib(), tok._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 1))
    try:
        got = tok.encode_batch(texts)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 0)
    bad = [i for i in range(len(texts)) if got[i] != exp[i]]
    assert not bad, "first differing string %d of %d" % (bad[0], len(texts))
    tok.close()


@pytest.mark.parametrize("host_presplit", [0, 1])
def test_bench_specials_batch_vs_oracle(host_presplit):
    """bench.py --specials 1 --pattern gpt2: the C2 corpus with special tokens spliced in (a
    separator at every string's end, ~1 more per KiB), cut to one launch; the occurrences found on
    the host, the pre-split on the device (fused) or on the host (C3 proper) -- id for id against
    the oracle's orc_encode_with_specials on every string."""
    import torch
    specials = {"<|endoftext|>": 50256, "<|fim_prefix|>": 50257, "<|fim_middle|>": 50258, "<|fim_suffix|>": 50259}
    buf, off = corpus.synth(BENCH_SEED, corpus.MIXED, 1_000_000, 1074, n_threads=THREADS)
    buf, off = corpus.splice_specials(buf, off, specials, per_kib=1.0, end_special=0, n_threads=THREADS)
    k = int(np.searchsorted(off, (1 << 30) - 64, side="right")) - 1
    buf, off = buf[:int(off[k])], off[:k + 1]
    tok = sa.Tokenizer(device=0)
    tok.merges = load_model_merges("bl32k.model")
    tok.pattern = sa.GPT2_PATTERN
    pos, ln, ids = corpus.find_specials(buf, off, specials, n_threads=THREADS)
    assert len(pos) > k
    dev = torch.device("cuda", 0)
    d_buf, d_off = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev)
    d_sp = tuple(torch.from_numpy(x).to(dev) for x in (pos, ln, ids))
    d_bits = None
    if host_presplit:
        bits, _ = corpus.presplit_specials(buf, off, pos, ln, _lib.SW_PAT_GPT2, n_threads=THREADS)
        d_bits = torch.from_numpy(bits.view(np.int64)).to(dev)
    g_ids, g_off = tok.encode_device(d_buf, d_off, d_bits=d_bits, d_specials=d_sp)
    got_ids, got_off = g_ids.cpu().numpy(), g_off.cpu().numpy()
    del d_buf, d_off, d_sp, d_bits, g_ids, g_off
    torch.cuda.empty_cache()
    exp_ids, exp_off = oracle.OracleModel(tok.merges).encode_batch_specials(buf, off, specials, oracle.PAT_GPT2,
                                                                            n_threads=THREADS)
    assert len(got_ids) == len(exp_ids), (len(got_ids), len(exp_ids), first_mismatch(got_ids, exp_ids))
    np.testing.assert_array_equal(got_off, exp_off)
    i = first_mismatch(got_ids, exp_ids)
    assert i == len(exp_ids), "first differing id at %d" % i
    tok.close()
