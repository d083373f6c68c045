"""Multi-rank path (shredword_amd/shard.py) on CPU: world_size 2 over gloo.

The per-rank GPU encode is stood in for by the oracle (this is a test of the partition and the
collective reassembly, not of the kernels); the reassembled batch must equal the committed
golden encode of the whole batch, bit for bit, on every rank."""
import os
import socket

import numpy as np
import pytest

from conftest import GOLD, load_model_merges

from shredword_amd import shard


def test_partition_is_byte_balanced_and_covers():
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 5000, size=1001)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    for world in (1, 2, 3, 8):
        parts = shard.partition(off, world)
        assert parts[0][0] == 0 and parts[-1][1] == len(lens)
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        sizes = [int(off[hi] - off[lo]) for lo, hi in parts]
        assert sum(sizes) == int(off[-1])
        assert max(sizes) - min(sizes) <= 2 * int(lens.max()) + 1


def test_partition_edge_cases():
    assert shard.partition(np.array([0], np.int64), 4) == [(0, 0)] * 4
    off = np.array([0, 10], np.int64)
    parts = shard.partition(off, 3)
    assert sum(hi - lo for lo, hi in parts) == 1
    off = np.array([0, 0, 0, 5, 5], np.int64)  # empty strings
    parts = shard.partition(off, 2)
    assert parts[0][0] == 0 and parts[-1][1] == 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, fixture, model, result_dir):
    import torch
    import torch.distributed as dist

    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = np.load(os.path.join(GOLD, fixture))
        buf, off = d["bytes"], d["off"]
        lo, hi = shard.partition(off, world)[rank]
        sub, sub_off = shard.shard_of(buf, off, lo, hi)
        om = oracle.OracleModel(load_model_merges(model))
        ids, ids_off = om.encode_batch(np.ascontiguousarray(sub), np.ascontiguousarray(sub_off), 0, n_threads=1)
        full_ids, full_off = shard.reassemble(torch.from_numpy(ids), torch.from_numpy(ids_off), None,
                                              torch.device("cpu"))
        ok = (np.array_equal(full_ids.numpy(), d["ids"]) and np.array_equal(full_off.numpy(), d["ids_off"]))
        # with caller bounds (no host synchronisation before the gathers): the same result
        b_ids, b_off = shard.reassemble(torch.from_numpy(ids), torch.from_numpy(ids_off), None, torch.device("cpu"),
                                        width=len(buf), width_s=len(off))
        shard.check_bounds()
        ok = ok and np.array_equal(b_ids.numpy(), d["ids"]) and np.array_equal(b_off.numpy(), d["ids_off"])
        # a bound below a rank's count is reported, never silently truncated
        try:
            shard.reassemble(torch.from_numpy(ids), torch.from_numpy(ids_off), None, torch.device("cpu"), width=1,
                             width_s=len(off))
            ok = False
        except RuntimeError:
            pass
        # 16-bit transport (every id of these tables < 65536): widened on arrival, the same
        w_ids, w_off = shard.reassemble(torch.from_numpy(ids), torch.from_numpy(ids_off), None, torch.device("cpu"),
                                        id_bits=16)
        ok = ok and np.array_equal(w_ids.numpy(), d["ids"]) and np.array_equal(w_off.numpy(), d["ids_off"])
        r16 = shard.reassemble(torch.from_numpy(ids), torch.from_numpy(ids_off), None, torch.device("cpu"),
                               concat=False, id_bits=16)
        ok = ok and r16[0].dtype == torch.int16
        # issued only (async_op): two batches in flight, then waited on -- both the whole batch
        t_ids, t_off = torch.from_numpy(ids), torch.from_numpy(ids_off)
        flights = [shard.reassemble(t_ids, t_off, None, torch.device("cpu"), concat=False, width=len(buf),
                                    width_s=len(off), id_bits=bits, async_op=True) for bits in (16, 32)]
        for works, res in flights:
            for w in works:
                w.wait()
            recv, counts, width, recv_o, n_strs, width_s = res
            got_ids, got_off, disp = [], [], 0
            for r in range(world):
                c, m = int(counts[r]), int(n_strs[r])
                got_ids.append(recv[r * width: r * width + c].to(torch.int32) & 0xFFFF)
                got_off.append(recv_o[r * width_s: r * width_s + m] + disp)
                disp += c
            got_off.append(torch.tensor([disp]))
            ok = ok and np.array_equal(torch.cat(got_ids).numpy(), d["ids"])
            ok = ok and np.array_equal(torch.cat(got_off).numpy(), d["ids_off"])
        # receive buffers kept across calls (bufs, as bench.py's step loop does): the second call
        # lands in the first call's tensors, and both compact to the whole batch
        keep, ptr = {}, None
        for rep in range(2):
            works, res = shard.reassemble(t_ids, t_off, None, torch.device("cpu"), concat=False, width=len(buf),
                                          width_s=len(off), id_bits=32, async_op=True, bufs=keep)
            for w in works:
                w.wait()
            ok = ok and (ptr is None or res[0].data_ptr() == ptr)
            ptr = res[0].data_ptr()
            out_ids, out_off = shard.compact(res, 32)
            ok = ok and np.array_equal(out_ids[:len(d["ids"])].numpy(), d["ids"])
            ok = ok and np.array_equal(out_off[:len(d["ids_off"])].numpy(), d["ids_off"])
        shard.check_bounds()
        try:  # async needs the bounds (no host synchronisation allowed)
            shard.reassemble(t_ids, t_off, None, torch.device("cpu"), concat=False, async_op=True)
            ok = False
        except ValueError:
            pass
        with open(os.path.join(result_dir, "rank%d" % rank), "w") as f:
            f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fixture,model", [("enc_bl32k_mixed.npz", "bl32k.model"),
                                           ("enc_toy500_ascii.npz", "toy500.model")])
def test_reassemble_gloo_world2(tmp_path, fixture, model):
    import torch.multiprocessing as mp

    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), fixture, model, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert open(tmp_path / ("rank%d" % r)).read() == "ok"
