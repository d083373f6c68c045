#!/usr/bin/env python3
"""Time sw_presplit_device alone on the bench corpus (HIP events on torch's stream), for each
library given (SHREDWORD_HIP_LIB is set per run by tools/gpu_ps_time.sh)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from shredword_amd import Tokenizer, _lib, corpus  # noqa: E402

pat = {"cl100k": 0, "gpt2": 1, "none": 2}[sys.argv[1] if len(sys.argv) > 1 else "cl100k"]
kname = sys.argv[2] if len(sys.argv) > 2 else "mixed"
kind = {"mixed": corpus.MIXED, "stress": corpus.STRESS, "ascii": corpus.ASCII}[kname]
buf, off = corpus.synth(1_000_003, kind, 1_000_000, 600 if kind == corpus.STRESS else 1074, n_threads=16)
n = int(off[-1])
dev = torch.device("cuda", 0)
tok = Tokenizer(device=0)
tok.merges = {(104, 105): 256}
h = tok._encoder()
L = _lib.lib()
d_buf = torch.from_numpy(buf).to(dev)
d_off = torch.from_numpy(off).to(dev)
d_bits = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev)


def run():
    _lib.check(L.sw_presplit_device(h, d_buf.data_ptr(), n, d_off.data_ptr(), len(off) - 1, pat, d_bits.data_ptr(),
                                    st.cuda_stream, None))


run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(5):
    run()
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
ok = ""
if os.environ.get("SHREDWORD_HIP_LIB") is None:
    exp, _ = corpus.presplit(buf[:50_000_000], off[:int(off.searchsorted(50_000_000, 'right'))], pat)
    got = d_bits.cpu().numpy().view("uint64")
    ok = " parity(first 50MB)=%s" % bool((got[:len(exp) - 1] == exp[:-1]).all())
print("%s %s: %.3f ms per presplit (incl. bitmap clear), %.1f GB/s%s" % (
    os.path.basename(os.environ.get("SHREDWORD_HIP_LIB", "default")), kname, ms, n / ms / 1e6, ok), flush=True)
