"""Document-sharded batch encode across the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on the MI355X node,
"gloo" for the CPU tests).  The batch is cut into contiguous string ranges balanced by bytes;
every rank encodes its range on its own device with no communication, and the only exchange
is the reassembly of the token-id buffers:
  1. all-gather of the per-rank token counts (int64);
  2. exclusive scan -> each rank's displacement in the global id buffer;
  3. all-gather of the id buffers, padded to the largest rank's count (one collective: on
     xGMI every GPU receives 7/8 of the ids over its 7 links at once);
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


def reassemble(local_ids, local_off, group=None, device=None, concat=True):
    """Collective reassembly of per-rank encodes (steps 1-4 above) on every rank.

    local_ids: torch int32 [>= local count] on `device`; local_off: torch int64 [m+1] with
    local_off[0] == 0.  Returns (ids int32 [total], off int64 [n+1]) for the whole batch, on
    `device`, identical on every rank.  concat=False skips the final copies and returns the
    gathered buffers as they landed: (ids [world * width], counts, width, offsets
    [world * width_s], string counts, width_s) -- rank r's ids start at r * width."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = device if device is not None else local_ids.device
    cnt = local_off[-1:].to(device=dev, dtype=torch.int64)
    counts = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, cnt, group=group)
    n_str = torch.tensor([local_off.numel() - 1], dtype=torch.int64, device=dev)
    n_strs = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(n_strs, n_str, group=group)
    counts_h = counts.cpu().tolist()
    n_strs_h = n_strs.cpu().tolist()
    width = max(max(counts_h), 1)
    c = int(counts_h[dist.get_rank(group)])
    if local_ids.numel() >= width and local_ids.dtype == torch.int32 and local_ids.device == dev:
        send = local_ids[:width]  # (slots past c are padding: never read)
    else:
        send = torch.zeros(width, dtype=torch.int32, device=dev)
        send[:c] = local_ids[:c].to(device=dev, dtype=torch.int32)
    recv = torch.empty(world * width, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(recv, send, group=group)
    width_s = max(max(n_strs_h), 1)
    m = int(n_strs_h[dist.get_rank(group)])
    if local_off.numel() >= width_s and local_off.dtype == torch.int64 and local_off.device == dev:
        send_o = local_off[:width_s]
    else:
        send_o = torch.zeros(width_s, dtype=torch.int64, device=dev)
        send_o[:m] = local_off[:m].to(device=dev, dtype=torch.int64)
    recv_o = torch.empty(world * width_s, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(recv_o, send_o, group=group)
    if not concat:
        return recv, counts_h, width, recv_o, n_strs_h, width_s
    ids, offs, disp = [], [], 0
    for r in range(world):
        ids.append(recv[r * width: r * width + counts_h[r]])
        offs.append(recv_o[r * width_s: r * width_s + n_strs_h[r]] + disp)
        disp += counts_h[r]
    offs.append(torch.tensor([disp], dtype=torch.int64, device=dev))
    return torch.cat(ids), torch.cat(offs)


def encode_sharded(tok, buf, str_off, chunk_bits_fn=None, group=None):
    """Encode the packed batch (buf, str_off) across the ranks of `group`: rank r encodes its
    byte-balanced string range with `tok` (a Tokenizer on this rank's GPU), then every rank
    gets the whole batch's ids via `reassemble`.  chunk_bits_fn(sub_buf, sub_off) may supply a
    pre-split bitmap for the sub-batch (default: the tokenizer's own host pre-split)."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = partition(str_off, world)[rank]
    sub, sub_off = shard_of(buf, str_off, lo, hi)
    bits = chunk_bits_fn(sub, sub_off) if chunk_bits_fn else None
    ids, off = tok.encode_packed(sub, sub_off, bits)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    return reassemble(torch.from_numpy(ids).to(dev), torch.from_numpy(off).to(dev), group, dev)
