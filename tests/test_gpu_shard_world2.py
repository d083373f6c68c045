"""The doc-sharded path as one piece in two processes on the MI355X box: world
size 2 over gloo, both ranks on device 0.  Each rank runs the real HIP encode
(Tokenizer.encode_packed, through the C-ABI) on its shard.partition range, shard.reassemble
gathers the ranks' ids (16- and 32-bit transport) and offsets, and the HIP reassembly pass
(shard.compact: offsets rebased, 16-bit ids widened) rebuilds the whole batch -- which must equal
the reference-generated golden ids on every rank.  bl50k puts ids >= 32768 through the int16
transport (negative on the wire, widened back).  The reference has no multi-device path, so the
golden ids of the whole batch are the oracle here."""
import os
import socket

import numpy as np
import pytest

from conftest import GOLD, load_model_merges

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, fixture, model, result_dir):
    import torch
    import torch.distributed as dist

    import shredword_amd as sa
    from shredword_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    msg = "ok"
    try:
        d = np.load(os.path.join(GOLD, fixture))
        buf, off = d["bytes"], d["off"]
        lo, hi = shard.partition(off, world)[rank]
        assert hi > lo, "every rank gets strings"
        sub, sub_off = shard.shard_of(buf, off, lo, hi)
        tok = sa.Tokenizer(device=0)
        tok.merges = load_model_merges(model)
        ids, ids_off = tok.encode_packed(np.ascontiguousarray(sub), np.ascontiguousarray(sub_off))
        t_ids, t_off = torch.from_numpy(ids), torch.from_numpy(ids_off)
        cpu, gpu = torch.device("cpu"), torch.device("cuda", 0)
        for bits in (16, 32):
            # exact-size reassembly (one host synchronisation for the sizes)
            full_ids, full_off = shard.reassemble(t_ids, t_off, None, cpu, id_bits=bits)
            if not (np.array_equal(full_ids.numpy(), d["ids"]) and np.array_equal(full_off.numpy(), d["ids_off"])):
                msg = "concat mismatch (%d-bit)" % bits
            # the bench's form: caller bounds, gathered buffers as landed, then the HIP pass
            res = shard.reassemble(t_ids, t_off, None, cpu, concat=False, width=len(buf), width_s=len(off),
                                   id_bits=bits)
            shard.check_bounds()
            if bits == 16 and int(d["ids"].max()) >= 32768 and int(res[0].min()) >= 0:
                msg = "16-bit transport did not wrap"
            dres = tuple(x.to(gpu) if isinstance(x, torch.Tensor) else x for x in res)
            c_ids, c_off = shard.compact(dres, bits)
            torch.cuda.synchronize()
            n, m = len(d["ids"]), len(d["ids_off"])
            if not (np.array_equal(c_ids[:n].cpu().numpy(), d["ids"])
                    and np.array_equal(c_off[:m].cpu().numpy(), d["ids_off"])):
                msg = "device reassembly mismatch (%d-bit)" % bits
        tok.close()
    except Exception as e:  # (reported through the result file)
        msg = "error: %r" % (e,)
    finally:
        with open(os.path.join(result_dir, "rank%d" % rank), "w") as f:
            f.write(msg)
        dist.destroy_process_group()


@pytest.mark.parametrize("fixture,model", [("enc_bl32k_mixed.npz", "bl32k.model"),
                                           ("enc_bl50k_stress.npz", "bl50k.model")])
def test_hip_encode_gloo_world2(tmp_path, fixture, model):
    import torch.multiprocessing as mp

    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), fixture, model, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert open(tmp_path / ("rank%d" % r)).read() == "ok", "rank %d" % r
