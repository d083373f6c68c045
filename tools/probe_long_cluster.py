"""Probe (GPU box): the device specials finder on long runs of self-overlapping specials (the
global-memory path's cluster walk) -- time and equality with the host finder."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import shredword_amd as sa  # noqa: E402
from shredword_amd import corpus  # noqa: E402
from conftest import load_model_merges  # noqa: E402

t = sa.Tokenizer(device=0)
t.merges = load_model_merges("bl32k.model")
for sp in ({"aa": 300, "aaa": 301}, {"aaa": 301, "aa": 300}):
    t.special_tokens = sp
    for n in [int(x) for x in sys.argv[1:]]:
        datas = [b"x" + b"a" * n + b"y", b"ab" * 100, b"a" * 7]
        off = np.zeros(len(datas) + 1, dtype=np.int64)
        np.cumsum([len(d) for d in datas], out=off[1:])
        buf = np.frombuffer(b"".join(datas), dtype=np.uint8).copy()
        d_buf = torch.from_numpy(buf).cuda()
        d_off = torch.from_numpy(off).cuda()
        torch.cuda.synchronize()
        t0 = time.time()
        pos, ln, ids, cnt, m = t.find_specials_device(d_buf, d_off, sync=True)
        torch.cuda.synchronize()
        dt = time.time() - t0
        hp, hl, hi = corpus.find_specials(buf, off, sp)
        ok = m == len(hp) and np.array_equal(pos[:m].cpu().numpy(), hp) and np.array_equal(ids[:m].cpu().numpy(), hi)
        print("specials %s run %d: %.3f s, %d occurrences, equal to host: %s" % (list(sp), n, dt, m, ok), flush=True)
t.close()
