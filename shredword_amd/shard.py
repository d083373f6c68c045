"""Document-sharded batch encode across the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on the MI355X node,
"gloo" for the CPU tests).  The batch is cut into contiguous string ranges balanced by bytes;
every rank encodes its range on its own device with no communication, and the only exchange
is the reassembly of the token-id buffers:
  1. all-gather of the per-rank token and string counts (int64, one collective);
  2. exclusive scan -> each rank's displacement in the global id buffer;
  3. all-gather of the id buffers, padded to the largest rank's count (one collective: on
     xGMI every GPU receives 7/8 of the ids over its 7 links at once), as 16-bit ids when the
     vocabulary fits (id_bits=16: half the bytes on the links; widened on arrival);
  4. per-string offsets rebased by the displacement and concatenated.

The reference has no multi-device path (its trainer is single-threaded, shredword/csrc/bpe);
this is the build's own layer, and the per-rank encode is exactly `Tokenizer.encode_packed`.
"""
import numpy as np


def partition(str_off, world):
    """Contiguous string ranges [(lo, hi)] for `world` ranks, cut at the byte quantiles of
    str_off (rank r gets about total/world bytes; a string is never split)."""
    str_off = np.asarray(str_off, dtype=np.int64)
    n = len(str_off) - 1
    if world < 1:
        raise ValueError("world must be >= 1")
    b0, b1 = int(str_off[0]), int(str_off[-1])
    cuts = [0]
    for r in range(1, world):
        target = b0 + (b1 - b0) * r // world
        s = int(np.searchsorted(str_off[:n + 1], target, side="left"))
        cuts.append(min(max(s, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_of(buf, str_off, lo, hi):
    """The packed sub-batch of strings [lo, hi): (bytes view, offsets rebased to 0)."""
    str_off = np.asarray(str_off, dtype=np.int64)
    a, b = int(str_off[lo]), int(str_off[hi])
    return buf[a:b], str_off[lo:hi + 1] - a


def reassemble(local_ids, local_off, group=None, device=None, concat=True, width=None, width_s=None, id_bits=32,
               async_op=False, bufs=None):
    """Collective reassembly of per-rank encodes (steps 1-4 above) on every rank.

    local_ids: torch int32 [>= local count] on `device` (or int16 holding each id's low 16 bits, e.g.
    from an encode with out_bits 16 -- sw_encode_ex -- when id_bits=16); local_off: torch int64 [m+1] with
    local_off[0] == 0.  Returns (ids int32 [total], off int64 [n+1]) for the whole batch, on
    `device`, identical on every rank.

    The per-rank token and string counts travel in ONE all-gather.  Sizing the padded gathers
    needs their maxima on the host -- one synchronisation -- unless the caller knows bounds:
    `width` >= every rank's token count and `width_s` >= every rank's string count (e.g. from an
    earlier step over the same batch); then nothing waits on the host, and a bound that was too
    small raises at the next synchronising call (check_bounds).
    concat=False skips the final copies and returns the gathered buffers as they landed:
    (ids [world * width], counts [world] on the device, width, offsets [world * width_s],
    string counts [world] on the device, width_s) -- rank r's ids start at r * width.
    id_bits=16 (every id < 65536, e.g. SW_INFO_IDS16): the ids travel as 16 bits; concat=True
    widens them to int32, concat=False returns them as int16 holding the low 16 bits (an id is
    `x & 0xFFFF` of the widened value).
    async_op=True (concat=False and both widths given): the collectives are only issued; returns
    (works, result) where result is concat=False's tuple, valid once every work in `works` has
    been waited on, in order (Work.wait(): with RCCL the caller's stream waits, the host does
    not; the last work folds the width check into the flag check_bounds reads).  The next
    batch's encode can run meanwhile -- the reassembly of batch k overlaps the encode of batch
    k + 1; local_ids / local_off must not be rewritten before the wait.
    bufs (with both widths): a dict the call keeps its device buffers in and reuses on the next
    call with the same dict -- a step loop then allocates nothing.  (A fresh 0.5 GB receive buffer
    per step went to hipMalloc while the previous one was still in use on the reassembly's
    stream, and that allocation waited for the device: the next encode could not be issued until
    the previous reassembly had finished.)  The caller must not reuse a dict before the
    previous call's buffers are consumed (one dict per batch in flight)."""
    import torch
    import torch.distributed as dist

    if async_op and (concat or width is None or width_s is None):
        raise ValueError("reassemble: async_op needs concat=False and both width bounds")
    world = dist.get_world_size(group)
    works, works_tail = [], []

    def gather(out, inp):
        w = dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
        if async_op:
            works.append(w)
    dev = device if device is not None else local_ids.device

    def buf(name, n, dtype):  # a device buffer, from `bufs` when the caller keeps them
        if bufs is None:
            return torch.empty(n, dtype=dtype, device=dev)
        b = bufs.get(name)
        if b is None or b.numel() != n or b.dtype != dtype or b.device != dev:
            b = bufs[name] = torch.empty(n, dtype=dtype, device=dev)
        return b
    mine = buf("mine", 2, torch.int64)
    mine[0:1] = local_off[-1:].to(device=dev, dtype=torch.int64)
    mine[1:2].fill_(local_off.numel() - 1)  # (a fill kernel: `mine[1] = n` copies from pageable host memory, synchronously)
    both = buf("both", 2 * world, torch.int64)
    gather(both, mine)  # [count_0, n_str_0, count_1, ...]
    counts, n_strs = both[0::2], both[1::2]
    if width is None or width_s is None:  # the one host synchronisation: the gathers' sizes
        h = both.cpu().tolist()
        width = max(max(h[0::2]), 1) if width is None else width
        width_s = max(max(h[1::2]), 1) if width_s is None else width_s
    elif not concat:  # (concat=True checks the counts itself below); async: once the gathers are waited on
        if async_op:
            works_tail.append(_BoundsCheck(counts, n_strs, int(width), int(width_s)))
        else:
            _note_bounds(counts, n_strs, int(width), int(width_s))
    width, width_s = int(width), int(width_s)
    if id_bits not in (16, 32):
        raise ValueError("id_bits must be 16 or 32")
    wide = id_bits == 32
    # the send buffer: the caller's ids as they are when they already have the transport's width
    # (16-bit: an encode with out_bits 16 -- no conversion pass), else converted
    want = torch.int32 if wide else torch.int16
    if local_ids.numel() >= width and local_ids.dtype == want and local_ids.device == dev:
        send = local_ids[:width]  # (slots past the count are padding: never read)
    else:
        send = torch.zeros(width, dtype=want, device=dev)
        k = min(width, local_ids.numel())
        # (16 bits: the low 16 bits of each id, two's-complement truncation of the int32 value)
        send[:k] = local_ids[:k].to(device=dev, dtype=torch.int32).to(want)
    recv = buf("recv", world * width, want)
    if wide:
        gather(recv, send)
    else:  # moved as bytes (RCCL and gloo have no 16-bit integer type; an all-gather only copies)
        gather(recv.view(torch.uint8), send.view(torch.uint8))
    m = local_off.numel() - 1
    if local_off.numel() >= width_s and local_off.dtype == torch.int64 and local_off.device == dev:
        send_o = local_off[:width_s]
    else:
        send_o = torch.zeros(width_s, dtype=torch.int64, device=dev)
        send_o[:min(m, width_s)] = local_off[:min(m, width_s)].to(device=dev, dtype=torch.int64)
    recv_o = buf("recv_o", world * width_s, torch.int64)
    gather(recv_o, send_o)
    if not concat:
        res = (recv, counts, width, recv_o, n_strs, width_s)
        return (works + works_tail, res) if async_op else res
    # the exact-size result needs the counts on the host (one synchronisation)
    ch, sh = counts.cpu().tolist(), n_strs.cpu().tolist()
    if max(ch) > width or max(sh) > width_s:
        raise RuntimeError("reassemble: a rank's count exceeds the given width bound")
    out_ids, out_off = compact((recv, counts, width, recv_o, n_strs, width_s), id_bits)
    return out_ids[:sum(ch)], out_off[:sum(sh) + 1]


def compact(res, id_bits=32, out_ids=None, out_off=None, stream=None):
    """Step 4 on the gathered buffers of reassemble(concat=False) `res`: the batch's contiguous
    int32 ids and rebased string offsets, without a host synchronisation.  Returns (out_ids,
    out_off), sized by the bounds (world * width ids, world * width_s + 1 offsets); the batch's
    ids are out_ids[:counts.sum()] and its offsets out_off[:n_strs.sum() + 1].

    On a GPU this is one HIP pass (sw_reassemble_device; `stream`: a torch stream, default the
    current one) -- 16-bit ids are widened on the way; on the CPU (gloo tests) torch ops."""
    import torch

    recv, counts, width, recv_o, n_strs, width_s = res
    world = counts.numel()
    dev = recv.device
    if out_ids is None:
        out_ids = torch.empty(max(world * width, 1), dtype=torch.int32, device=dev)
    if out_off is None:
        out_off = torch.empty(world * width_s + 1, dtype=torch.int64, device=dev)
    if out_ids.numel() < world * width or out_off.numel() < world * width_s + 1:
        raise ValueError("compact: output buffers below the bounds")
    if dev.type == "cuda":
        from . import _lib
        stream = stream or torch.cuda.current_stream(dev)
        for t in (recv, recv_o, counts, n_strs, out_ids, out_off):  # (buffers the caller may drop before the pass ran)
            t.record_stream(stream)
        with torch.cuda.stream(stream):  # (the counts are strided views of the counts all-gather)
            counts, n_strs = counts.contiguous(), n_strs.contiguous()
            _lib.check(_lib.lib().sw_reassemble_device(recv.data_ptr() if recv.numel() else None, int(id_bits),
                                                       counts.data_ptr(), int(width),
                                                       recv_o.data_ptr() if recv_o.numel() else None,
                                                       n_strs.data_ptr(), int(width_s), int(world),
                                                       out_ids.data_ptr(), out_off.data_ptr(), stream.cuda_stream))
        return out_ids, out_off
    ch = [min(max(int(c), 0), width) for c in counts.tolist()]
    sh = [min(max(int(c), 0), width_s) for c in n_strs.tolist()]
    disp = sdisp = 0
    for r in range(world):
        blk = recv[r * width: r * width + ch[r]].to(torch.int32)
        out_ids[disp: disp + ch[r]] = (blk & 0xFFFF) if id_bits == 16 else blk
        out_off[sdisp: sdisp + sh[r]] = recv_o[r * width_s: r * width_s + sh[r]] + disp
        disp += ch[r]
        sdisp += sh[r]
    out_off[sdisp] = disp
    return out_ids, out_off


# Width bounds given to reassemble are checked without a host synchronisation: each call folds
# "some count exceeded its bound" into one flag tensor per device (constant memory however many
# calls run); check_bounds() reads the flags (one synchronisation) and clears them.
_bound_flags = {}


def _note_bounds(counts, n_strs, width, width_s):
    import torch
    over = torch.logical_or((counts > width).any(), (n_strs > width_s).any())
    flag = _bound_flags.get(counts.device)
    if flag is None:
        _bound_flags[counts.device] = over.clone()
    else:
        flag.logical_or_(over)


class _BoundsCheck:
    """The bounds check of an async reassembly, as the last entry of its works: its wait() runs
    after the gathers' waits, so the comparison is ordered after the counts have landed."""

    def __init__(self, counts, n_strs, width, width_s):
        self.args = (counts, n_strs, width, width_s)

    def wait(self):
        if self.args is not None:
            _note_bounds(*self.args)
            self.args = None
        return True


def check_bounds():
    """Raise if a width bound given to reassemble (concat=False) since the last call was exceeded by
    an actual count; a too-small bound truncates the gathered ids, so call this once per batch (or
    per group of batches) before using their results.  Synchronises with the devices: the flags
    may have been written on any stream (an async reassembly folds them on the stream its works
    were waited on), so the whole device is synchronised before they are read."""
    import torch
    for dev in _bound_flags:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    bad = [str(dev) for dev, flag in _bound_flags.items() if bool(flag.item())]
    _bound_flags.clear()
    if bad:
        raise RuntimeError("reassemble: a rank's count exceeded the width bounds (devices %s)" % ", ".join(bad))


def encode_sharded(tok, buf, str_off, chunk_bits_fn=None, group=None):
    """Encode the packed batch (buf, str_off) across the ranks of `group`: rank r encodes its
    byte-balanced string range with `tok` (a Tokenizer on this rank's GPU), then every rank
    gets the whole batch's ids via `reassemble`.

    With the nccl (RCCL) backend the rank's shard is uploaded once and encoded, pre-split
    included, on device buffers (Tokenizer.encode_device); the ids stay on the device through
    the all-gather.  chunk_bits_fn(sub_buf, sub_off) may supply a host pre-split bitmap.  With
    gloo (CPU tests) the host-buffer path encode_packed is used."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = partition(str_off, world)[rank]
    sub, sub_off = shard_of(buf, str_off, lo, hi)
    bits = chunk_bits_fn(sub, sub_off) if chunk_bits_fn else None
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        d_buf = torch.from_numpy(np.ascontiguousarray(sub) if len(sub) else np.zeros(1, np.uint8)).to(dev)
        d_off = torch.from_numpy(np.ascontiguousarray(sub_off)).to(dev)
        d_bits = torch.from_numpy(bits.view(np.int64)).to(dev) if bits is not None else None
        ids, off = tok.encode_device(d_buf, d_off, d_bits)
        return reassemble(ids, off, group, dev, id_bits=16 if tok.ids16 else 32)
    ids, off = tok.encode_packed(sub, sub_off, bits)
    dev = torch.device("cpu")
    return reassemble(torch.from_numpy(ids).to(dev), torch.from_numpy(off).to(dev), group, dev,
                      id_bits=16 if tok.ids16 else 32)
