"""Which call of the world-1 RCCL gather blocks the host?  Each candidate runs while the GPU is
busy (torch.cuda._sleep) and its host time is printed (GPU box; diagnostic)."""
import os
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
off = torch.arange(1001, dtype=torch.int64, device=dev)
ids = torch.zeros(1 << 20, dtype=torch.int16, device=dev)
recv = torch.empty_like(ids)
both = torch.empty(2, dtype=torch.int64, device=dev)
dist.all_gather_into_tensor(recv.view(torch.uint8), ids.view(torch.uint8))  # (warm)
torch.cuda.synchronize()


def timed(name, fn):
    torch.cuda._sleep(200_000_000)
    t = time.perf_counter()
    r = fn()
    print("%-40s %8.3f ms" % (name, (time.perf_counter() - t) * 1e3), flush=True)
    torch.cuda.synchronize()
    return r


mine = torch.empty(2, dtype=torch.int64, device=dev)
timed("mine[0:1] = off[-1:]", lambda: mine.__setitem__(slice(0, 1), off[-1:].to(device=dev, dtype=torch.int64)))
timed("mine[1] = int", lambda: mine.__setitem__(1, 1000))
timed("all_gather int64 async", lambda: dist.all_gather_into_tensor(both, mine, async_op=True))
timed("all_gather uint8 view async", lambda: dist.all_gather_into_tensor(recv.view(torch.uint8), ids.view(torch.uint8), async_op=True))
w = timed("all_gather int64 async (keep)", lambda: dist.all_gather_into_tensor(both, mine, async_op=True))
timed("work.wait()", lambda: w.wait())
timed("torch.empty", lambda: torch.empty(1 << 20, dtype=torch.int16, device=dev))
s2 = torch.cuda.Stream(dev)
timed("side.wait_stream", lambda: s2.wait_stream(torch.cuda.current_stream(dev)))
dist.destroy_process_group()
