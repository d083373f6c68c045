"""Probe (GPU box): per-call latency of small sw_encode_device launches (a kernel trace of the
steady state: run under rocprofv3 --kernel-trace --stats)."""
import ctypes
import os
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

nb_target = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
t = sa.Tokenizer(device=0)
t.merges = load_model_merges("bl32k.model")
buf, off = corpus.synth(5, corpus.MIXED, 2000, 1074)
k = max(1, int(np.searchsorted(off, nb_target, side="right")) - 1)
nb = int(off[k])
dev = torch.device("cuda", 0)
d_buf = torch.from_numpy(buf[:nb].copy()).to(dev)
d_off = torch.from_numpy(off[:k + 1].copy()).to(dev)
d_out = torch.empty(nb + 16, dtype=torch.int32, device=dev)
d_oo = torch.empty(k + 1, dtype=torch.int64, device=dev)
L, h = _lib.lib(), t._encoder()
stream = torch.cuda.current_stream(dev).cuda_stream
ts = []
for i in range(reps):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    _lib.check(L.sw_encode_device(h, d_buf.data_ptr(), nb, d_off.data_ptr(), k, None, d_out.data_ptr(), d_oo.data_ptr(),
                                  stream, None))
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    ts.append((t1 - t0, time.perf_counter() - t0))
ts = ts[3:]
print("bytes %d strings %d: host enqueue %.1f us, call+sync %.1f us (medians of %d)" % (
    nb, k, 1e6 * sorted(a for a, _ in ts)[len(ts) // 2], 1e6 * sorted(b for _, b in ts)[len(ts) // 2], len(ts)))
t.close()
