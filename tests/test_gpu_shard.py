"""The multi-GPU path on the MI355X box: shard.encode_sharded over RCCL (torch.distributed
backend "nccl") at world size 1 with the HIP encoder on device buffers, against the
reference-generated golden ids; and the reassembly with caller width bounds (no host
synchronisation before the gathers)."""
import os
import socket

import numpy as np
import pytest

import shredword_amd as sa
from shredword_amd import _lib, shard
from conftest import GOLD, load_model_merges

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_world1():
    import torch
    import torch.distributed as dist
    if _lib.lib().sw_device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu must run on the MI355X box")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("fixture,model", [("enc_bl32k_mixed.npz", "bl32k.model"),
                                           ("enc_toy500_ascii.npz", "toy500.model"),
                                           ("enc_bl50k_stress.npz", "bl50k.model")])
def test_encode_sharded_rccl_world1(nccl_world1, fixture, model):
    import torch
    d = np.load(os.path.join(GOLD, fixture))
    tok = sa.Tokenizer(device=0)
    tok.merges = load_model_merges(model)
    ids, off = shard.encode_sharded(tok, d["bytes"], d["off"])
    assert ids.device.type == "cuda" and off.device.type == "cuda"
    np.testing.assert_array_equal(off.cpu().numpy(), d["ids_off"])
    np.testing.assert_array_equal(ids.cpu().numpy(), d["ids"])
    # the gathered buffers with caller bounds (the bench's step): rank 0's ids at offset 0
    d_buf = torch.from_numpy(d["bytes"]).cuda()
    d_off = torch.from_numpy(d["off"]).cuda()
    l_ids, l_off = tok.encode_device(d_buf, d_off)
    recv, counts, width, recv_o, n_strs, width_s = shard.reassemble(l_ids, l_off, None, torch.device("cuda", 0),
                                                                    concat=False, width=len(d["bytes"]),
                                                                    width_s=len(d["off"]))
    shard.check_bounds()
    n = int(counts[0].item())
    np.testing.assert_array_equal(recv[:n].cpu().numpy(), d["ids"])
    np.testing.assert_array_equal(recv_o[:len(d["off"]) - 1].cpu().numpy(), d["ids_off"][:-1])
    # 16-bit transport over RCCL (the bench's step when every id fits): low 16 bits as landed (bl50k:
    # ids >= 32768 cross the int16 cast as negative values), widened by the HIP reassembly pass
    assert tok.ids16
    r16 = shard.reassemble(l_ids, l_off, None, torch.device("cuda", 0), concat=False, width=len(d["bytes"]),
                           width_s=len(d["off"]), id_bits=16)
    shard.check_bounds()
    assert r16[0].dtype == torch.int16
    np.testing.assert_array_equal((r16[0][:n].to(torch.int32) & 0xFFFF).cpu().numpy(), d["ids"])
    if int(d["ids"].max()) >= 32768:
        assert int(r16[0][:n].min().item()) < 0  # (the wrap-around is exercised)
    c_ids, c_off = shard.compact(r16, 16)
    np.testing.assert_array_equal(c_ids[:n].cpu().numpy(), d["ids"])
    np.testing.assert_array_equal(c_off[:len(d["off"])].cpu().numpy(), d["ids_off"])
    ids16, off16 = shard.reassemble(l_ids, l_off, None, torch.device("cuda", 0), id_bits=16)  # (concat=True)
    np.testing.assert_array_equal(ids16.cpu().numpy(), d["ids"])
    np.testing.assert_array_equal(off16.cpu().numpy(), d["ids_off"])
    # the bench's overlapped step: batch k's gathers issued (RCCL stream), batch k+1 encoded into
    # the other buffers meanwhile, then every gather waited on (the stream waits, not the host)
    outs = [(torch.empty(len(d["bytes"]), dtype=torch.int32, device="cuda"),
             torch.empty(len(d["off"]), dtype=torch.int64, device="cuda")) for _ in range(2)]
    flights = []
    for o_ids, o_off in outs:
        tok.encode_device(d_buf, d_off, d_out=o_ids, d_out_off=o_off)
        flights.append(shard.reassemble(o_ids, o_off, None, torch.device("cuda", 0), concat=False,
                                        width=len(d["bytes"]), width_s=len(d["off"]), id_bits=16, async_op=True))
    for works, res in flights:
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        assert int(res[1][0].item()) == n
        np.testing.assert_array_equal((res[0][:n].to(torch.int32) & 0xFFFF).cpu().numpy(), d["ids"])
        np.testing.assert_array_equal(res[3][:len(d["off"]) - 1].cpu().numpy(), d["ids_off"][:-1])
    shard.check_bounds()
    tok.close()


@pytest.mark.parametrize("id_bits", [16, 32])
def test_reassemble_device_kernel(id_bits):
    """sw_reassemble_device (shard.compact) on synthetic gathered buffers of 5 ranks, one of them
    empty and one filling its width exactly: ids widened from the low 16 bits (values >= 32768
    included), offsets rebased by the ids before each rank, the total as the last offset; the
    padding is never read into the output."""
    import torch
    rng = np.random.default_rng(11)
    world, width, width_s = 5, 3001, 41
    counts = np.array([1234, 0, 3001, 17, 2900], np.int64)
    n_strs = np.array([40, 0, 41, 1, 7], np.int64)
    ids = [rng.integers(0, 65536 if id_bits == 16 else 1 << 31, size=c) for c in counts]
    recv = np.full(world * width, 0x5A5A if id_bits == 16 else -7, np.int64)
    recv_o = np.full(world * width_s, -99, np.int64)
    for r in range(world):
        recv[r * width: r * width + counts[r]] = ids[r]
        o = np.sort(rng.integers(0, counts[r] + 1, size=n_strs[r]))
        if n_strs[r]:
            o[0] = 0
        recv_o[r * width_s: r * width_s + n_strs[r]] = o
    dev = torch.device("cuda", 0)
    t_recv = torch.from_numpy(recv.astype(np.uint16).view(np.int16) if id_bits == 16 else recv.astype(np.int32)).to(dev)
    res = (t_recv, torch.from_numpy(counts).to(dev), width, torch.from_numpy(recv_o).to(dev),
           torch.from_numpy(n_strs).to(dev), width_s)
    out_ids, out_off = shard.compact(res, id_bits)
    torch.cuda.synchronize()
    exp_ids = np.concatenate(ids).astype(np.int64)
    exp_off, disp = [], 0
    for r in range(world):
        exp_off.append(recv_o[r * width_s: r * width_s + n_strs[r]] + disp)
        disp += counts[r]
    exp_off = np.concatenate(exp_off + [np.array([disp])])
    np.testing.assert_array_equal(out_ids[:len(exp_ids)].cpu().numpy().astype(np.int64) & (0xFFFF if id_bits == 16 else -1),
                                  exp_ids)
    assert int(out_ids[:len(exp_ids)].min().item()) >= 0
    np.testing.assert_array_equal(out_off[:len(exp_off)].cpu().numpy(), exp_off)
    # the CPU (gloo) form of the same pass gives the same
    cpu = tuple(x.cpu() if hasattr(x, "cpu") else x for x in res)
    c_ids, c_off = shard.compact(cpu, id_bits)
    np.testing.assert_array_equal(c_ids[:len(exp_ids)].numpy(), out_ids[:len(exp_ids)].cpu().numpy())
    np.testing.assert_array_equal(c_off[:len(exp_off)].numpy(), exp_off)
