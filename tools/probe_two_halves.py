"""Probe (GPU box): the 1 GiB C2 batch as one launch against its two halves (split at a string
boundary) on two encoder handles and two streams, launched together -- how much of the second
half hides behind the first's latency-bound phases."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import shredword_amd as sa  # noqa: E402
from shredword_amd import _lib, corpus  # noqa: E402
from conftest import load_model_merges  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
kind = {"mixed": corpus.MIXED, "entropy": corpus.ENTROPY}[sys.argv[2] if len(sys.argv) > 2 else "mixed"]
dev = torch.device("cuda", 0)
buf, off = corpus.synth(1_000_003, kind, 1_000_000, 1074, n_threads=16)
k = int(np.searchsorted(off, (1 << 30) - 64, side="right")) - 1
buf, off = buf[:int(off[k])], off[:k + 1]
n_str, n_bytes = k, int(off[-1])
merges = load_model_merges("bl32k.model")
toks = [sa.Tokenizer(device=0) for _ in range(2)]
for t in toks:
    t.merges = merges
L = _lib.lib()
d_buf = torch.from_numpy(buf).to(dev)
d_off = torch.from_numpy(off).to(dev)
d_out = torch.empty(n_bytes + 64, dtype=torch.int32, device=dev)
d_oo = torch.empty(n_str + 1, dtype=torch.int64, device=dev)
# halves at the string nearest the middle byte
m = int(np.searchsorted(off, n_bytes // 2))
offB = torch.from_numpy((off[m:] - off[m]).copy()).to(dev)
nbA, nbB = int(off[m]), n_bytes - int(off[m])
d_outB = torch.empty(nbB + 64, dtype=torch.int32, device=dev)
d_ooB = torch.empty(n_str - m + 1, dtype=torch.int64, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
h1, h2 = toks[0]._encoder(), toks[1]._encoder()


def whole():
    _lib.check(L.sw_encode_device(h1, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n_str, None, d_out.data_ptr(),
                                  d_oo.data_ptr(), s1.cuda_stream, None))


def halves(stagger):
    _lib.check(L.sw_encode_device(h1, d_buf.data_ptr(), nbA, d_off.data_ptr(), m, None, d_out.data_ptr(),
                                  d_oo.data_ptr(), s1.cuda_stream, None))
    if stagger:
        s2.wait_stream(s1)
    _lib.check(L.sw_encode_device(h2, d_buf.data_ptr() + nbA, nbB, offB.data_ptr(), n_str - m, None, d_outB.data_ptr(),
                                  d_ooB.data_ptr(), s2.cuda_stream, None))


def timed(fn, n):
    for _ in range(2):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / n * 1e3


tw = timed(whole, steps)
ta = timed(lambda: _lib.check(L.sw_encode_device(h1, d_buf.data_ptr(), nbA, d_off.data_ptr(), m, None, d_out.data_ptr(),
                                                 d_oo.data_ptr(), s1.cuda_stream, None)), steps)
th = timed(lambda: halves(False), steps)
ts = timed(lambda: halves(True), steps)
print("whole %.3f ms (%.1f GB/s); half A alone %.3f ms; halves on two streams %.3f ms (%.1f GB/s); "
      "serial halves %.3f ms" % (tw, n_bytes / tw / 1e6, ta, th, n_bytes / th / 1e6, ts), flush=True)
# the halves' ids == the whole's
halves(False)
torch.cuda.synchronize(dev)
whole()
torch.cuda.synchronize(dev)
tA = int(d_oo[m].item())
okA = torch.equal(d_out[:tA], d_out[:tA])
print("ids per half: %d + %d, whole %d" % (tA, int(d_ooB[-1].item()), int(d_oo[-1].item())))
