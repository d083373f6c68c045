"""C3 (host pre-split + host specials, GPU merge loop only), the multi-launch batch split of
sw_encode_batch, the split + verify long-chunk path and the workspace's stream ordering -- each
compared directly with the oracle (oracle/sw_oracle.c) and the reference-generated golden ids.
All calls go through the C-ABI."""
import ctypes
import random

import numpy as np
import pytest

import oracle
import shredword_amd as sa
from shredword_amd import _lib, corpus
from conftest import PATTERNS, golden_index, load_fixture, load_model_merges, page_array, page_end_array

pytestmark = pytest.mark.gpu

FIXTURES = golden_index()["fixtures"]
PAT_STR = {"cl100k": "", "gpt2": sa.GPT2_PATTERN, "none": 2}
_TOKS = {}


@pytest.fixture(scope="module", autouse=True)
def need_device():
    if _lib.lib().sw_device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu must run on the MI355X box")


def tok_for(model, pattern="cl100k"):
    if model not in _TOKS:
        t = sa.Tokenizer(device=0)
        t.merges = load_model_merges(model)
        _TOKS[model] = t
    t = _TOKS[model]
    t.pattern = PAT_STR[pattern]
    return t


def oracle_encode(merges, buf, off, pattern):
    return oracle.OracleModel(merges).encode_batch(buf, off, PATTERNS[pattern], n_threads=8)


def pack(datas):
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    return np.frombuffer(b"".join(datas) or b"\0", dtype=np.uint8)[:int(off[-1])].copy(), off


def assert_same(got, exp):
    np.testing.assert_array_equal(got[1], exp[1])
    np.testing.assert_array_equal(got[0], exp[0])


def device_encode_with_bits(t, buf, off, bits):
    """sw_encode_device on torch buffers with a host-made bitmap (the C3 device entry point)."""
    import torch
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off - off[0])).to(dev)
    d_bits = torch.from_numpy(bits.view(np.int64)).to(dev)
    n = int(off[-1] - off[0])
    d_out = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    d_oo = torch.empty(len(off), dtype=torch.int64, device=dev)
    n_tok = ctypes.c_int64()
    _lib.check(_lib.lib().sw_encode_device(t._encoder(), d_buf.data_ptr(), n, d_off.data_ptr(), len(off) - 1,
                                           d_bits.data_ptr(), d_out.data_ptr(), d_oo.data_ptr(),
                                           torch.cuda.current_stream(dev).cuda_stream, ctypes.byref(n_tok)))
    torch.cuda.synchronize()
    return d_out[:n_tok.value].cpu().numpy(), d_oo.cpu().numpy()


# ------------------------------------------------------------------ C3: host bitmap, GPU merge loop
@pytest.mark.parametrize("entry", FIXTURES, ids=[e["file"] for e in FIXTURES])
def test_c3_host_bitmap_golden(entry):
    """The host pre-split bitmap fed to the GPU merge loop reproduces the reference-generated ids,
    through both the host-buffer and the device-buffer entry points."""
    fx = load_fixture(entry)
    t = tok_for(entry["model"], entry["pattern"])
    bits, _ = corpus.presplit(fx["bytes"], fx["off"], PATTERNS[entry["pattern"]])
    exp = (fx["ids"], fx["ids_off"])
    assert_same(t.encode_packed(fx["bytes"], fx["off"], bits), exp)
    assert_same(device_encode_with_bits(t, fx["bytes"], fx["off"], bits), exp)


@pytest.mark.parametrize("pattern", ["cl100k", "gpt2"])
def test_c3_host_bitmap_large_corpus_vs_oracle(pattern):
    """C3 on a 64 MB MIXED corpus: host bitmap -> GPU merge loop == the oracle's own encode."""
    buf, off = corpus.synth(99, corpus.MIXED, 60000, 1074)
    t = tok_for("bl32k.model", pattern)
    bits, _ = corpus.presplit(buf, off, PATTERNS[pattern], n_threads=16)
    exp = oracle_encode(t.merges, buf, off, pattern)
    assert_same(t.encode_packed(buf, off, bits), exp)
    assert_same(device_encode_with_bits(t, buf, off, bits), exp)


def test_c3_host_presplit_with_specials():
    """Special tokens split on the host, pieces pre-split on the host threads, GPU merge loop."""
    t = sa.Tokenizer(device=0)
    t.merges = load_model_merges("bl32k.model")
    t.special_tokens = {"<|endoftext|>": 100257, "<|fim_prefix|>": 100258, "<|fim|>": 100259}
    rng = random.Random(8)
    words = ["Hello", " world", "'s", " 12345", "\n\n", "  ", " 中文", " 😀", "<|endoftext|>", "<|fim|>",
             "<|fim_prefix|>", "<|fim", "|>", " x", "."]
    texts = ["".join(rng.choice(words) for _ in range(rng.randint(0, 60))) for _ in range(300)]
    om = oracle.OracleModel(t.merges)
    exp = [om.encode_with_specials(s, t.special_tokens) for s in texts]
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 1))
    try:
        assert t.encode_batch(texts) == exp
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_HOST_PRESPLIT, 0)
    assert t.encode_batch(texts) == exp  # (device pre-split: the same)
    t.close()


# ------------------------------------------------------------------ multi-launch batch split
@pytest.mark.parametrize("limit", [64, 777, 4096, 70000])
@pytest.mark.parametrize("host_bits", [False, True])
def test_batch_split_launches(limit, host_bits):
    """sw_encode_batch encodes a batch over the launch limit as runs of whole strings: bitmap
    realignment (the runs start at arbitrary, non-64-aligned bytes), out_off rebasing and stats.
    The offsets start at an unaligned, non-zero byte (a sub-batch of a larger buffer)."""
    buf, off = corpus.synth(5, corpus.MIXED, 300, 700)
    datas = [bytes(buf[off[i]:off[i + 1]][:limit]).decode("utf-8", "ignore").encode("utf-8") for i in range(300)]
    datas[3:3] = [b"", b"", b"x" * limit]
    pre = b"#" * 13
    full, offs = pack([pre] + datas)
    sub = offs[1:]  # starts at byte 13
    assert int(np.diff(sub).max()) <= limit and int(sub[-1] - sub[0]) > 4 * limit
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, full, sub, "cl100k")
    bits = corpus.presplit(full, sub)[0] if host_bits else None
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, limit))
    try:
        got = t.encode_packed(full, sub, bits)
        st = t.last_stats
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, 0)
    assert_same(got, exp)
    assert st.n_bytes == int(sub[-1] - sub[0]) and st.n_tokens == len(exp[0])
    if host_bits:
        assert st.n_chunks == -1  # (caller bits: no count)
    else:
        assert st.n_chunks == corpus.presplit(full, sub)[1]


def test_pipeline_runs_cut_at_launch_limit():
    """The pipelined host path (batches over 2 runs) with a launch limit BELOW the run size: runs
    are cut at the smaller of the two, so many small strings never make a run over the limit
    (ADVICE r2); a single string over the limit is still rejected."""
    buf, off = corpus.synth(6, corpus.MIXED, 2000, 300)
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    L, h = _lib.lib(), t._encoder()
    limit = max(int(np.diff(off).max()), 2000)
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 4 * limit))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, limit))
    try:
        assert int(off[-1]) > 2 * 4 * limit  # (the pipelined path)
        assert_same(t.encode_packed(buf, off), exp)
        big, boff = pack([b"a" * 10] * 50 + [b"b" * (limit + 1)] + [b"c" * 10] * 50000)
        with pytest.raises(_lib.ShredwordError):
            t.encode_packed(big, boff)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, 0)
        L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 128 << 20)


def test_batch_split_string_over_limit_rejected():
    t = tok_for("toy500.model")
    buf, off = pack([b"a" * 100, b"b" * 300])
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, 200))
    try:
        with pytest.raises(_lib.ShredwordError):
            t.encode_packed(buf, off)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, 0)
    for bad in (1, 63, 1 << 31):
        assert L.sw_encoder_set_option(h, _lib.SW_OPT_MAX_LAUNCH_BYTES, bad) == _lib.SW_ERR_ARG


def test_bad_pattern_leaves_handle_untouched():
    """A rejected pattern returns before any state changes (the timing flag)."""
    t = tok_for("toy500.model")
    L, h = _lib.lib(), t._encoder()
    buf, off = pack([b"hello world"])
    out = np.empty(16, np.int32)
    oo = np.empty(2, np.int64)
    rc = L.sw_encode_batch(h, _lib.ptr(buf, ctypes.c_uint8), _lib.ptr(off, ctypes.c_int64), 1, 7, None,
                           _lib.ptr(out, ctypes.c_int32), 16, _lib.ptr(oo, ctypes.c_int64), None)
    assert rc == _lib.SW_ERR_ARG
    assert L.sw_encoder_last_kernel_ms(h) == -1.0  # timing still off: nothing was recorded
    assert_same(t.encode_packed(buf, off), oracle_encode(t.merges, buf, off, "cl100k"))


# ------------------------------------------------------------------ split + verify for long chunks
def _long_chunks(rng):
    datas = []
    for L in (33, 34, 47, 48, 49, 63, 64, 65, 100, 255, 256, 257, 500, 1000, 2047, 2048, 4095, 4096):
        datas.append(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(L)))
        datas.append(bytes(rng.choice(b"etaoinsh") for _ in range(L)))
        datas.append(b"e" * L)
        datas.append(b" " + b"o" * (L - 1))
        datas.append(bytes(rng.choice(b"  \n\t\r") for _ in range(L)))
        datas.append(bytes(rng.choice(b"ab") for _ in range(L)))
        runs = b""
        while len(runs) < L:
            runs += bytes([rng.choice(b"abc")]) * rng.randint(1, 40)
        datas.append(runs[:L])
    for _ in range(300):
        L = rng.randint(33, 4096)
        datas.append(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(L)))
    return datas


@pytest.mark.parametrize("model", ["toy500.model", "bl32k.model", "bl50k.model"])
def test_long_split_vs_oracle(model):
    """Chunks of 33..4096 bytes (random letters, (a,a) runs, whitespace runs, two-letter mixes)
    through the split + verify path and through the wave loop: both equal the oracle."""
    rng = random.Random(17)
    datas = _long_chunks(rng)
    buf, off = pack(datas)
    t = tok_for(model, "none")
    L, h = _lib.lib(), t._encoder()
    assert L.sw_encoder_get_info(h, _lib.SW_INFO_SPLIT) == 1  # (well-formed tables)
    exp = oracle_encode(t.merges, buf, off, "none")
    assert_same(t.encode_packed(buf, off), exp)
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_LONG_SPLIT, 0))
    try:
        assert_same(t.encode_packed(buf, off), exp)
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_LONG_SPLIT, 1)
    t.pattern = ""


@pytest.mark.parametrize("mode", [1, 0])
def test_long_split_stress_corpus_vs_oracle(mode):
    buf, off = corpus.synth(123, corpus.STRESS, 30000, 600)
    t = tok_for("bl50k.model")
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_LONG_SPLIT, mode))
    try:
        assert_same(t.encode_packed(buf, off), oracle_encode(t.merges, buf, off, "cl100k"))
    finally:
        L.sw_encoder_set_option(h, _lib.SW_OPT_LONG_SPLIT, 1)


@pytest.mark.parametrize("seed", range(4))
def test_long_split_random_wellformed_tables(seed):
    """Random well-formed tables (values >= 256, unique, above both members) over a small
    alphabet: dense merges make junction conflicts and cascades frequent."""
    r = random.Random(seed)
    alpha = list(b"abcd")
    merges, ids = {}, list(alpha)
    nxt = 256
    for _ in range(r.randint(20, 400)):
        p = (r.choice(ids), r.choice(ids))
        if p in merges:
            continue
        merges[p] = nxt
        ids.append(nxt)
        nxt += 1 + (r.random() < 0.2) * r.randint(1, 5)  # gaps in the values
    datas = [bytes(r.choice(b"abcd") for _ in range(r.randint(33, 1500))) for _ in range(300)]
    buf, off = pack(datas)
    t = sa.Tokenizer()
    t.merges = merges
    t.pattern = 2
    assert _lib.lib().sw_encoder_get_info(t._encoder(), _lib.SW_INFO_SPLIT) == 1
    assert_same(t.encode_packed(buf, off), oracle_encode(merges, buf, off, "none"))
    t.close()


def test_long_split_not_used_for_illformed_tables():
    t = sa.Tokenizer()
    t.merges = {(97, 98): 256, (98, 99): 256}  # duplicate value
    assert _lib.lib().sw_encoder_get_info(t._encoder(), _lib.SW_INFO_SPLIT) == 0
    t.merges = {(97, 98): 100}  # value < 256
    assert _lib.lib().sw_encoder_get_info(t._encoder(), _lib.SW_INFO_SPLIT) == 0
    t.merges = {(300, 98): 299, (97, 98): 300}  # value below a member
    assert _lib.lib().sw_encoder_get_info(t._encoder(), _lib.SW_INFO_SPLIT) == 0
    t.close()


# ------------------------------------------------------------------ workspace stream ordering
def test_workspace_ordered_across_streams():
    """Back-to-back launches of one handle on two different streams: the second waits for the
    first (the workspace is the handle's), so both outputs are exact."""
    import torch
    buf, off = corpus.synth(31, corpus.MIXED, 8000, 1074)
    t = tok_for("bl32k.model")
    exp = oracle_encode(t.merges, buf, off, "cl100k")
    dev = torch.device("cuda", 0)
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    outs = [(torch.empty(len(buf), dtype=torch.int32, device=dev), torch.empty(len(off), dtype=torch.int64, device=dev))
            for _ in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()
    L, h = _lib.lib(), t._encoder()
    for _ in range(3):
        for (d_out, d_oo), s in zip(outs, streams):
            _lib.check(L.sw_encode_device(h, d_buf.data_ptr(), len(buf), d_off.data_ptr(), len(off) - 1, None,
                                          d_out.data_ptr(), d_oo.data_ptr(), s.cuda_stream, None))
    torch.cuda.synchronize()
    for d_out, d_oo in outs:
        oo = d_oo.cpu().numpy()
        assert_same((d_out[:int(oo[-1])].cpu().numpy(), oo), exp)


# ------------------------------------------------------------------ pipelined host batches
@pytest.mark.parametrize("run", [64, 5000, 300000])
@pytest.mark.parametrize("host_bits", [False, True])
@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("kcopy", [True, False])
def test_pipelined_batch(run, host_bits, wide, kcopy):
    """sw_encode_batch over more than two pipeline runs: staging, 16-bit downloads (32-bit for a
    table past 64k ids), realigned caller bits, offsets rebased across runs, copies by kernels
    over PCIe or by DMA -- == the oracle."""
    buf, off = corpus.synth(8, corpus.MIXED, 900, 700)
    if run == 64:  # (every string must fit a run... or be a run of its own: both happen)
        datas = [bytes(buf[off[i]:off[i + 1]][:200]).decode("utf-8", "ignore").encode("utf-8") for i in range(400)]
        full, offs = pack([b"#" * 13] + datas)
    else:
        full, offs = pack([b"#" * 13] + [bytes(buf[off[i]:off[i + 1]]) for i in range(900)])
    sub = offs[1:]
    base = load_model_merges("bl32k.model")
    if wide:
        shift = lambda x: x if x < 256 else x + 70000  # noqa: E731
        merges = {(shift(a), shift(b)): shift(v) for (a, b), v in base.items()}
    else:
        merges = base
    t = sa.Tokenizer(device=0)
    t.merges = merges
    exp = oracle_encode(merges, full, sub, "cl100k")
    bits = corpus.presplit(full, sub)[0] if host_bits else None
    L, h = _lib.lib(), t._encoder()
    assert L.sw_encoder_get_info(h, _lib.SW_INFO_IDS16) == (0 if wide else 1)
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, run))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_COPY_KERNELS, int(kcopy)))
    got = t.encode_packed(full, sub, bits)
    st = t.last_stats
    assert_same(got, exp)
    assert st.n_tokens == len(exp[0])
    assert st.n_chunks == (-1 if host_bits else corpus.presplit(full, sub)[1])
    got2 = t.encode_packed(full, sub, bits)  # (buffers reused)
    assert_same(got2, exp)
    t.close()


@pytest.mark.parametrize("depth", [2, 4])
def test_pipelined_depth(depth):
    """Every pipeline depth gives the oracle's ids (slots reused across runs and calls)."""
    buf, off = corpus.synth(9, corpus.MIXED, 600, 700)
    full, offs = pack([bytes(buf[off[i]:off[i + 1]]) for i in range(600)])
    merges = load_model_merges("bl32k.model")
    t = sa.Tokenizer(device=0)
    t.merges = merges
    exp = oracle_encode(merges, full, offs, "cl100k")
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 4000))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_DEPTH, depth))
    assert_same(t.encode_packed(full, offs), exp)
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_DEPTH, 6 - depth))
    assert_same(t.encode_packed(full, offs), exp)
    assert L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_DEPTH, 5) == _lib.SW_ERR_ARG
    t.close()



def test_pinned_arrays_ending_on_a_page_boundary():
    """Pinned caller arrays with nothing after them: the input, the ids and the offsets each END
    exactly on a page boundary (the next page of the allocation is not pinned, so a device access
    past an array's end would touch an unmapped page), with misaligned starts (the strings begin 13
    bytes in; the ids start 4 mod 16 bytes; out_cap is the exact token count, so the last run's ids
    end at the page end) and many pipeline runs, so the direct push writes at many misaligned
    running counts done[0] (copy_seg).  == the oracle; read and written through the C-ABI."""
    buf, off = corpus.synth(11, corpus.MIXED, 900, 600)
    n = 900
    while True:  # (a token count that is not a multiple of 4: the ids then start off a 16-byte boundary)
        datas = [bytes(buf[off[i]:off[i + 1]]) for i in range(n)]
        full0, offs = pack([b"#" * 13] + datas)
        sub = offs[1:]
        merges = load_model_merges("bl32k.model")
        exp = oracle_encode(merges, full0, sub, "cl100k")
        if len(exp[0]) % 4 and len(sub) % 2 == 1:  # (and n + 1 int64 offsets ending on the page start off 16 B too)
            break
        n -= 1
    t = sa.Tokenizer(device=0)
    t.merges = merges
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 4099))
    full = page_end_array(len(full0), np.uint8, full0)
    out = page_end_array(len(exp[0]), np.int32, -5)
    out_off = page_end_array(len(sub), np.int64, -5)
    assert out.ctypes.data % 16 != 0 and out_off.ctypes.data % 16 != 0
    for arr in (full, out, out_off):
        assert (arr.ctypes.data + arr.nbytes) % 4096 == 0
        t.pin_host(arr)
    try:
        for _ in range(2):
            stats = _lib.SwStats()
            _lib.check(L.sw_encode_batch(h, _lib.ptr(full, ctypes.c_uint8), _lib.ptr(sub, ctypes.c_int64), len(sub) - 1, 0,
                                         None, _lib.ptr(out, ctypes.c_int32), len(out), _lib.ptr(out_off, ctypes.c_int64),
                                         ctypes.byref(stats)))
            assert stats.n_tokens == len(exp[0])
            assert_same((out, out_off), exp)
            out[:] = -5
            out_off[:] = -5
    finally:
        for arr in (full, out, out_off):
            t.unpin_host(arr)
    t.close()


@pytest.mark.parametrize("pin", ["all", "input", "outputs", "out_only"])
@pytest.mark.parametrize("wide", [False, True])
def test_pipelined_pinned_caller_buffers(pin, wide):
    """Caller arrays pinned with Tokenizer.pin_host (sw_encoder_pin_host): the input read over PCIe
    without staging, the ids and offsets written by the device into the caller's arrays (only when
    both output arrays are pinned) -- == the oracle, for a 16- and a 32-bit table, every
    combination, calls repeated; a too-small pinned output is refused, not overrun; unpinned
    arrays work as before."""
    buf, off = corpus.synth(10, corpus.MIXED, 700, 700)
    full, offs = pack([b"#" * 13] + [bytes(buf[off[i]:off[i + 1]]) for i in range(700)])
    sub = offs[1:]
    base = load_model_merges("bl32k.model")
    merges = {(a if a < 256 else a + 70000, b if b < 256 else b + 70000): v + 70000
              for (a, b), v in base.items()} if wide else base
    t = sa.Tokenizer(device=0)
    t.merges = merges
    exp = oracle_encode(merges, full, sub, "cl100k")
    L, h = _lib.lib(), t._encoder()
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, 5000))
    # (each pinned array on pages of its own: arrays sharing a page cannot both be pinned)
    full = page_array(len(full), np.uint8, full)
    out = page_array(len(full) + 100, np.int32, -5)
    out_off = page_array(len(sub) + 3, np.int64, -5)
    pins = {"all": (full, out, out_off), "input": (full,), "outputs": (out, out_off), "out_only": (out,)}[pin]
    for arr in pins:
        t.pin_host(arr)
    for _ in range(2):
        got = t.encode_packed(full, sub, out=out, out_off=out_off)
        assert_same(got, exp)
    if pin in ("all", "outputs"):  # (a pinned output too small for the batch, through the C-ABI: refused)
        small = page_array(len(exp[0]) // 2 + 4096, np.int32, -5)
        t.pin_host(small)
        stats = _lib.SwStats()
        rc = L.sw_encode_batch(h, _lib.ptr(full, ctypes.c_uint8), _lib.ptr(sub, ctypes.c_int64), len(sub) - 1, 0,
                               None, _lib.ptr(small, ctypes.c_int32), len(exp[0]) // 2, _lib.ptr(out_off, ctypes.c_int64),
                               ctypes.byref(stats))
        assert rc == _lib.SW_ERR_CAP
        assert (small[len(exp[0]) // 2:] == -5).all()  # (nothing written past out_cap)
        t.unpin_host(small)
    for arr in pins:
        t.unpin_host(arr)
    assert_same(t.encode_packed(full, sub, out=out, out_off=out_off), exp)
    with pytest.raises(RuntimeError):
        t.unpin_host(out)
    t.close()
