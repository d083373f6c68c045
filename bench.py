#!/usr/bin/env python3
"""Batched BPE encode throughput on MI355X -- the BASELINE.json metric.

One step = one pass of the encode hot path over one batch already resident in HBM: the whole
sw_encode_device pipeline (k_presplit, k_tile_strings, k_classify, queue scan/scatter,
k_merge_bucket x4, k_merge_long*, k_tile_count + scan, k_compact, k_string_offsets):
  N=1  BASELINE configs[1]: 1 GiB synthetic MIXED UTF-8, 1M strings (mean 1074 B), 32k-merge
       byte-level table; the full path (C2): cl100k pre-split on the GPU, merge loop, id
       compaction.  --presplit host gives configs[2] (C3: host pre-split, GPU merge loop only).
  N>1  configs[3]: every rank encodes its own 1 GiB corpus (seed + rank; doc-sharded), then the
       token-id buffers are reassembled on every rank with an RCCL all-gather (padded to the
       largest rank's count; 16-bit ids when every id fits) -- weak scaling, the gather is inside
       the step (--no-gather: without it); batch k's gather runs on RCCL's stream beside batch
       k+1's encode, every gather waited on before the clock stops (--no-overlap: one after the
       other).
Prints ONE JSON line (rank 0).  Launch for N>1:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
      --master-port P bench.py --gpus N
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues of this process (read by HIP at its first call, which comes later): the step
# uses up to five streams -- the launch stream, the two merge forks, RCCL's and the reassembly's.
# With HIP's default of 4 two of them shared one queue and ran in launch order, so the next
# batch's encode queued behind the previous batch's reassembly (profiles/r3f_gw1_trace.md).
os.environ["GPU_MAX_HW_QUEUES"] = "8"

SPECIALS = {"<|endoftext|>": 50256, "<|fim_prefix|>": 50257, "<|fim_middle|>": 50258, "<|fim_suffix|>": 50259}
LAUNCH_LIMIT = (1 << 30) - 64  # bytes of one sw_encode_device launch
METRIC = "encoded MB/s (input bytes) + Mtokens/s at 32k merges, 1/2/4/8 MI355X vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=["c3", "c5"],
                    help="c3: 1 GiB MIXED + 32k merges (configs[1]/[2]); c5: stress, 50k merges")
    ap.add_argument("--corpus", default=None, choices=["mixed", "stress", "entropy", "ascii"],
                    help="override the config's corpus kind (entropy: low repetition, most multi-token chunks "
                         "distinct -- the merge loop without the memoisation's help)")
    ap.add_argument("--specials", type=float, default=0.0,
                    help="C3 with special tokens: insert <|endoftext|> at every string's end and about this many "
                         "others per KiB at random code-point boundaries; found (and, with --presplit host, "
                         "pre-split) on the host threads, timed apart from the GPU step; the batch is cut to "
                         "the 2^30 - 64-byte launch limit")
    ap.add_argument("--specials-device", action="store_true",
                    help="with --specials: the occurrences are found on the device inside the timed step "
                         "(sw_find_specials_device, the count left on the device for sw_encode_device_ex) "
                         "instead of on the host threads before it")
    ap.add_argument("--strings", type=int, default=None)
    ap.add_argument("--mean-len", type=int, default=None)
    ap.add_argument("--pattern", default="cl100k", choices=["cl100k", "gpt2"])
    ap.add_argument("--presplit", default="device", choices=["device", "host"],
                    help="device: C2 full path (pre-split inside the step); host: C3 (bitmap made on the host)")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the RCCL reassembly")
    ap.add_argument("--gather-world1", action="store_true",
                    help="testing: N=1 with an RCCL process group and the reassembly in the step")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: each step's reassembly completes before the next step's encode")
    ap.add_argument("--cpu-sample-mb", type=float, default=320.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--small-steps", type=int, default=20,
                    help="rank 0, N=1: per-call latency of ~64 KiB and ~1 MiB prefixes through the same handle after "
                         "the big launches (0: skip)")
    ap.add_argument("--e2e-steps", type=int, default=2,
                    help="N=1: also time host buffers -> host buffers (PCIe-inclusive, reported beside value)")
    ap.add_argument("--threads", type=int, default=0,
                    help="host threads for corpus/pre-split and the all-cores CPU baseline (0: every usable core)")
    ap.add_argument("--no-dedupe", action="store_true",
                    help="A/B only: every queued chunk runs its own merge loop (same results)")
    ap.add_argument("--dedupe-slots", type=int, default=0, help="A/B only: cap the dedupe table (power of two)")
    ap.add_argument("--no-dedupe-exact", action="store_true", help="A/B only: fingerprint keys for every chunk")
    ap.add_argument("--no-merge-streams", action="store_true", help="A/B only: merge kernels one after another")
    ap.add_argument("--staged-heads", type=int, default=0, choices=[0, 1, 2],
                    help="A/B only: result heads staged by k_tile_count (0 automatic, 1 always, 2 never)")
    ap.add_argument("--no-fused", action="store_true",
                    help="A/B only: the device pre-split as its own kernel before k_classify (same results)")
    ap.add_argument("--pipe-dma", action="store_true", help="A/B only: e2e pipeline copies by DMA, not kernels")
    ap.add_argument("--pipe-depth", type=int, default=0, help="A/B only: e2e pipeline runs in flight (2..4)")
    ap.add_argument("--pipe-run-mb", type=int, default=0, help="A/B only: e2e pipeline run size (MiB)")
    ap.add_argument("--no-chunk-table", action="store_true",
                    help="every chunk runs the merge loop (results identical; see DESIGN.md)")
    return ap.parse_args()


def host_cpu():
    """(usable cores of this process, machine CPUs, CPU model name)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")  # (the GPU box states its CPU share this way)
    if share and share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return usable, os.cpu_count(), model


def main():
    args = parse()
    usable_cores, machine_cpus, cpu_model = host_cpu()
    if args.threads <= 0:
        args.threads = min(usable_cores, 64)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", args.gpus))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))

    import torch
    import torch.distributed as dist

    from shredword_amd import Tokenizer, _lib, corpus, shard

    use_dist = world > 1 or args.gather_world1
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    c5 = args.config == "c5"
    kind = corpus.STRESS if c5 else corpus.MIXED
    corpus_name = args.corpus or ("stress" if c5 else "mixed")
    if args.corpus:
        kind = {"mixed": corpus.MIXED, "stress": corpus.STRESS, "entropy": corpus.ENTROPY, "ascii": corpus.ASCII}[args.corpus]
    n_str = args.strings or (1_000_000 if not c5 else 1_000_000)
    mean = args.mean_len or (1074 if not c5 else 600)
    model = "bl50k.model" if c5 else "bl32k.model"
    pat = {"cl100k": _lib.SW_PAT_CL100K, "gpt2": _lib.SW_PAT_GPT2}[args.pattern]

    t = time.time()
    buf, off = corpus.synth(1_000_003 + rank, kind, n_str, mean, n_threads=args.threads)
    specials = None
    sp_host = None
    t_split = None
    if args.specials > 0:  # C3 with special tokens (the corpus carries their text)
        specials = dict(SPECIALS)
        buf, off = corpus.splice_specials(buf, off, specials, per_kib=args.specials, end_special=0,
                                          n_threads=args.threads)
        k = int(np.searchsorted(off, LAUNCH_LIMIT, side="right")) - 1  # (one launch: cut whole strings)
        buf, off = buf[:int(off[k])], off[:k + 1]
        n_str = k
    host_ps = args.presplit == "host"
    sp_device = bool(specials) and args.specials_device
    if sp_device and host_ps:
        raise SystemExit("--specials-device needs the device pre-split (the host pre-split needs host occurrences)")
    t_data = time.time() - t
    t = time.time()
    if specials:
        sp_host = corpus.find_specials(buf, off, specials, n_threads=args.threads)
    if host_ps:
        bits, n_chunks = (corpus.presplit_specials(buf, off, sp_host[0], sp_host[1], pat, n_threads=args.threads)
                          if specials else corpus.presplit(buf, off, pat, n_threads=args.threads))
    else:
        bits, n_chunks = None, -1
    t_split = time.time() - t
    t_prep = t_data + t_split
    n_bytes = int(off[-1])

    tok = Tokenizer(device=local)
    tok.load(os.path.join(ROOT, "tests", "golden", model))
    tok.pattern = pat
    L = _lib.lib()
    h = tok._encoder()
    _lib.check(L.sw_encoder_reserve(h, n_bytes, n_str))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_CHUNK_TABLE, 0 if args.no_chunk_table else 1))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE, 0 if args.no_dedupe else 1))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_SLOTS, args.dedupe_slots))
    if args.no_dedupe_exact:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_DEDUPE_EXACT, 0))
    if args.no_merge_streams:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_MERGE_STREAMS, 0))
    if args.staged_heads:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_STAGED_HEADS, args.staged_heads))
    if args.no_fused:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_FUSED_PRESPLIT, 0))
    if args.pipe_dma:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_COPY_KERNELS, 0))
    if args.pipe_depth:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_DEPTH, args.pipe_depth))
    if args.pipe_run_mb:
        _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PIPE_RUN_BYTES, args.pipe_run_mb << 20))
    _lib.check(L.sw_encoder_set_option(h, _lib.SW_OPT_PATTERN, pat))

    cap = torch.tensor([n_bytes], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(cap, op=dist.ReduceOp.MAX)
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_bits = torch.from_numpy(bits.view(np.int64)).to(dev) if host_ps else None
    gather = use_dist and not args.no_gather
    id_bits = 16 if tok.ids16 else 32  # (the ids cross xGMI as 16 bits when every id fits: SURVEY.md 8(e))
    # the multi-GPU step encodes straight into the transport's width (SW_OPT_OUT_BITS 16: no
    # conversion pass before the gather, half the output bytes); N=1 writes int32
    out16 = gather and id_bits == 16 and not specials
    d_out = torch.empty(int(cap.item()), dtype=torch.int16 if out16 else torch.int32, device=dev)
    d_oo = torch.empty(n_str + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    # per-call choices (sw_encode_ex): the caller's bitmap (None: device pre-split, C2), the ids'
    # width, the special-token occurrences found on the host (uploaded once, like the bitmap)
    ex = _lib.SwEncodeEx(d_bits.data_ptr() if host_ps else None, 16 if out16 else 32, None, None, None, 0)
    d_sp = None
    if sp_device:  # found on the device inside the step: arrays for the worst case, the count on the device
        st_sp, keep_sp = _lib.specials_struct(specials)
        _lib.check(L.sw_encoder_set_specials(h, ctypes.byref(st_sp)))
        cap_sp = n_bytes // min(len(k.encode()) for k in specials if k) + 1
        d_sp = (torch.empty(cap_sp, dtype=torch.int64, device=dev), torch.empty(cap_sp, dtype=torch.int32, device=dev),
                torch.empty(cap_sp, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int64, device=dev))
        ex.sp_pos, ex.sp_len, ex.sp_id, ex.n_sp = d_sp[0].data_ptr(), d_sp[1].data_ptr(), d_sp[2].data_ptr(), cap_sp
        ex.d_n_sp = d_sp[3].data_ptr()
    elif specials:
        d_sp = tuple(torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in sp_host)
        ex.sp_pos, ex.sp_len, ex.sp_id, ex.n_sp = d_sp[0].data_ptr(), d_sp[1].data_ptr(), d_sp[2].data_ptr(), len(sp_host[0])

    plain = not out16 and not specials  # (sw_encode_device: what an A/B build of an earlier revision has)

    def encode_into(o_ids, o_off, n_tok_ptr=None):
        if sp_device:
            _lib.check(L.sw_find_specials_device(h, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n_str,
                                                 d_sp[0].data_ptr(), d_sp[1].data_ptr(), d_sp[2].data_ptr(), cap_sp,
                                                 d_sp[3].data_ptr(), stream, None))
        if plain:
            _lib.check(L.sw_encode_device(h, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n_str,
                                          d_bits.data_ptr() if host_ps else None, o_ids.data_ptr(), o_off.data_ptr(),
                                          stream, n_tok_ptr))
        else:
            _lib.check(L.sw_encode_device_ex(h, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n_str, ctypes.byref(ex),
                                             o_ids.data_ptr(), o_off.data_ptr(), stream, n_tok_ptr))

    def encode(n_tok_ptr=None):
        encode_into(d_out, d_oo, n_tok_ptr)

    if not host_ps and not specials:  # chunk count for the report (outside the timed region)
        tmp_bits = torch.empty((n_bytes + 63) // 64, dtype=torch.int64, device=dev)
        c = ctypes.c_int64()
        _lib.check(L.sw_presplit_device(h, d_buf.data_ptr(), n_bytes, d_off.data_ptr(), n_str, pat,
                                        tmp_bits.data_ptr(), stream, ctypes.byref(c)))
        n_chunks = int(c.value)
        del tmp_bits

    n_tok_c = ctypes.c_int64()
    encode(ctypes.byref(n_tok_c))
    n_tok = int(n_tok_c.value)
    sp_dev_ok = None
    if sp_device:  # (the device finder's occurrences == the host threads', outside the timed region)
        nd = int(d_sp[3].item())
        sp_dev_ok = bool(nd == len(sp_host[0]) and np.array_equal(d_sp[0][:nd].cpu().numpy(), sp_host[0])
                         and np.array_equal(d_sp[2][:nd].cpu().numpy(), sp_host[2]))

    # the gathers' widths: every rank's counts are the same every step (same corpus), so the
    # maxima are taken once here and the timed step has no host synchronisation
    width = width_s = None
    if gather:
        mx = torch.tensor([n_tok, n_str], dtype=torch.int64, device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        width, width_s = int(mx[0].item()), int(mx[1].item()) + 1

    # N>1: batch k's reassembly overlaps batch k+1's encode.  The all-gathers run on RCCL's stream;
    # the compaction into the batch's contiguous int32 ids and rebased offsets (SURVEY.md 8(e) step 4,
    # sw_reassemble_device) runs on a side stream that waits for them; two sets of output buffers,
    # and a set is rewritten only after the side stream's event for it (a stream wait, no host
    # round trip)
    overlap = gather and not args.no_overlap
    outs = [(d_out, d_oo)]
    if overlap:
        outs.append((torch.empty_like(d_out), torch.empty_like(d_oo)))
    finals = []
    if gather:  # the reassembled batch: world * width ids, world * width_s + 1 offsets
        finals = [(torch.empty(world * width, dtype=torch.int32, device=dev),
                   torch.empty(world * width_s + 1, dtype=torch.int64, device=dev)) for _ in outs]
    side = torch.cuda.Stream(dev) if gather else None
    gbufs = [{} for _ in outs]  # the gathers' receive buffers, one set per batch in flight (no allocation in the step)
    done_ev = [None for _ in outs]
    n_step = [0]
    host_t = {"encode": 0.0, "gathers": 0.0, "reassembly": 0.0}  # (SW_BENCH_HOST_TIMES=1: host time per call)

    def step():
        slot = n_step[0] % len(outs)
        n_step[0] += 1
        h0 = time.perf_counter()
        if done_ev[slot] is not None:
            torch.cuda.current_stream(dev).wait_event(done_ev[slot])
            done_ev[slot] = None
        o_ids, o_off = outs[slot]
        encode_into(o_ids, o_off)
        h1 = time.perf_counter()
        host_t["encode"] += h1 - h0
        if not gather:
            return
        # steps 1-3: one counts all-gather, padded id and offset all-gathers (RCCL)
        works, res = shard.reassemble(o_ids, o_off, None, dev, concat=False, width=width, width_s=width_s,
                                      id_bits=id_bits, async_op=True, bufs=gbufs[slot])
        h2 = time.perf_counter()
        host_t["gathers"] += h2 - h1
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # step 4 once the gathers have landed
            for w in works:
                w.wait()
            shard.compact(res, id_bits, finals[slot][0], finals[slot][1])
            ev = torch.cuda.Event()
            ev.record(side)
        done_ev[slot] = ev
        host_t["reassembly"] += time.perf_counter() - h2
        if not overlap:
            torch.cuda.current_stream(dev).wait_event(ev)
            done_ev[slot] = None

    def finish():  # every issued reassembly complete before the clock stops (the caller's stream)
        for k, ev in enumerate(done_ev):
            if ev is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
                done_ev[k] = None

    for _ in range(args.warmup):
        step()
    finish()
    _lib.check(L.sw_encoder_set_timing(h, 1))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for k in host_t:
        host_t[k] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_issued = time.perf_counter()
    finish()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if os.environ.get("SW_BENCH_HOST_TIMES") == "1":
        sys.stderr.write("host ms per step: %s, all issued after %.3f ms of %.3f\n" % (
            {k: round(v * 1e3 / args.steps, 3) for k, v in host_t.items()}, (t_issued - t0) * 1e3 / args.steps,
            (t1 - t0) * 1e3 / args.steps))
    if world > 1:
        dist.barrier()
    k_ms = L.sw_encoder_last_kernel_ms(h)
    try:  # (the dominant kernel alone, HIP events on the launch stream; absent from older A/B builds)
        cls_ms = L.sw_encoder_last_classify_ms(h)
    except AttributeError:
        cls_ms = -1.0
    _lib.check(L.sw_encoder_set_timing(h, 0))
    reassembly_ok = None
    if gather:
        shard.check_bounds()
        # the last step's reassembled batch holds this rank's own encode at its displacement, and its
        # offsets end at the batch total
        last = (n_step[0] - 1) % len(outs)
        mine = torch.tensor([n_tok, n_str], dtype=torch.int64, device=dev)
        all_c = torch.empty(2 * world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(all_c, mine)
        cs, ss = all_c[0::2].tolist(), all_c[1::2].tolist()
        disp, sdisp = sum(cs[:rank]), sum(ss[:rank])
        f_ids, f_off = finals[last]
        o_ids, o_off = outs[last]
        mine_ids = (o_ids[:n_tok].to(torch.int32) & 0xFFFF) if out16 else o_ids[:n_tok]
        reassembly_ok = bool(torch.equal(f_ids[disp:disp + n_tok], mine_ids)
                             and torch.equal(f_off[sdisp:sdisp + n_str] - disp, o_off[:n_str])
                             and int(f_off[sum(ss)].item()) == sum(cs))
        ok_t = torch.tensor([1 if reassembly_ok else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)  # (every rank's check)
        reassembly_ok = bool(ok_t.item())

    # what the launches did: chunks settled without the merge loop, distinct merged after dedupe
    cnt4 = (ctypes.c_int64 * 4)()
    _lib.check(L.sw_encoder_last_counts(h, cnt4))
    l_chunks, l_refs, l_distinct = int(cnt4[0]), int(cnt4[1]), int(cnt4[2])
    rates = {"chunks": l_chunks, "to_merge_loop": l_refs, "merged_distinct": l_distinct,
             "settled_without_merge_loop": round(1 - l_refs / max(l_chunks, 1), 4),
             "dedupe_distinct_fraction": round(l_distinct / max(l_refs, 1), 4),
             "note": "settled = single bytes + whole-chunk-table hits; distinct = merge loops actually run "
                     "per chunk sent to the merge loop (the in-launch dedupe shares the rest)"}
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    totals = torch.tensor([n_bytes, n_tok, n_str, n_chunks], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(totals, op=dist.ReduceOp.SUM)
    sec = float(elapsed.item())
    all_bytes, all_tok, all_str, all_chunks = (float(x) for x in totals.tolist())
    ms_step = sec / args.steps * 1e3
    value = all_bytes * args.steps / sec / 1e6

    # roofline of the encode pipeline (all sw_encode_device kernels, HIP events), rank-local, per launch
    # bytes in + ids out + offsets in/out (+ the bitmap when it comes from the host, C3)
    # (ids written as 16 bits by the N>1 step, out16: 2 bytes each)
    b_algo = n_bytes + (2 if out16 else 4) * n_tok + 16 * (n_str + 1) + ((n_bytes + 7) // 8 if host_ps else 0)
    if sp_device:  # (the finder's kernels precede the encode's timing events: the whole step instead)
        k_ms = ms_step
    achieved = b_algo / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None
    # traffic: HBM bytes per launch from the committed PMC profile of this same workload, if any
    traffic, traffic_x2, traffic_src, counters, dom_prof = None, None, None, None, None
    try:  # (one entry per workload, written by tools/summarize_prof.py from that workload's PMC run)
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            tj = json.load(f)
        want = {"n_bytes": n_bytes, "merges": len(tok.merges), "pattern": args.pattern,
                "chunk_table": not args.no_chunk_table, "dedupe": not args.no_dedupe, "presplit": args.presplit,
                "corpus": corpus_name, "specials": args.specials,
                "specials_found": "device" if sp_device else "host"}
        for ent in tj.get("entries", []):
            if all(ent.get(k) == v for k, v in want.items()):
                traffic, traffic_src = int(ent["traffic_bytes_per_launch"]), ent["source"]
                traffic_x2 = int(ent.get("traffic_bytes_per_launch_x2", 0)) or None
                counters = ent.get("counters")
                dom_prof = ent.get("dominant")
    except (OSError, ValueError, KeyError):
        pass
    roofline = {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
                "traffic": traffic, "traffic_x2": traffic_x2,
                "traffic_over_algo": round(traffic / b_algo, 2) if traffic else None,
                "traffic_x2_over_algo": round(traffic_x2 / b_algo, 2) if traffic_x2 else None,
                "traffic_note": "HBM-side FETCH_SIZE + WRITE_SIZE per launch from the committed PMC profile; "
                                "traffic raw, traffic_x2 with FETCH doubled (gfx950 wide-read rule, an upper "
                                "bound here)",
                "traffic_source": traffic_src, "kernel": ("sw_encode_device pipeline (k_presplit..k_string_offsets)" if not host_ps else "sw_encode_device pipeline (k_tile_strings..k_string_offsets)"),
                "kernel_ms": round(k_ms, 4),
                "algo_bytes_per_launch": int(b_algo),
                "counters": counters}
    # the dominant kernel's own roofline: the classification reads the input once,
    # writes one 4-byte slot per chunk and writes (device pre-split) or reads (caller's bitmap) n/8
    # bytes of chunk-start bitmap; its time from HIP events around it on the launch stream, live
    dom_algo = n_bytes + 4 * l_chunks + (n_bytes + 7) // 8
    dom = {"kernel": "k_classify" if host_ps else "k_split_classify",
           "algo_bytes_per_launch": int(dom_algo),
           "algo_note": "input bytes + 4 B slot per chunk + n/8 bitmap (written by the fused pre-split, read with "
                        "a caller's bitmap)",
           "kernel_ms": round(cls_ms, 4) if cls_ms > 0 else None,
           "achieved": round(dom_algo / (cls_ms * 1e-3) / 1e9, 2) if cls_ms > 0 else None,
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(dom_algo / (cls_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if cls_ms > 0 else None,
           "share_of_pipeline": round(cls_ms / k_ms, 3) if cls_ms > 0 and k_ms > 0 else None}
    if dom_prof:  # (the committed PMC profile of this workload: the same kernel's trace time and bytes)
        dom["trace_ms"] = dom_prof.get("avg_ms")
        dom["traffic"] = dom_prof.get("traffic_bytes")
        dom["traffic_over_algo"] = round(dom_prof["traffic_bytes"] / dom_algo, 2) if dom_prof.get("traffic_bytes") else None
        dom["fetch_bytes"] = dom_prof.get("fetch_bytes")
        dom["write_bytes"] = dom_prof.get("write_bytes")
        dom["traffic_source"] = traffic_src
    roofline["dominant"] = dom

    # small launches after the big ones (rank 0, N=1): the same handle -- its dedupe table as the
    # 1 GiB launches left it (grown, on the low-repetition corpus) -- on prefixes of the batch of about
    # 64 KiB and 1 MiB through the device entry, each call synchronised: the per-call latency a small
    # batch pays (the table clear runs in k_edges only when its grid covers the table)
    small = None
    if rank == 0 and world == 1 and args.small_steps > 0 and plain and not gather and not host_ps:
        small = {}
        for target in (1 << 16, 1 << 20):
            k = max(1, int(np.searchsorted(off, target, side="right")) - 1)
            nb = int(off[k])
            ts = []
            for _ in range(args.small_steps + 2):
                torch.cuda.synchronize(dev)
                t_s = time.perf_counter()
                _lib.check(L.sw_encode_device(h, d_buf.data_ptr(), nb, d_off.data_ptr(), k, None, d_out.data_ptr(),
                                              d_oo.data_ptr(), stream, None))
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t_s)
            ts = sorted(ts[2:])
            small[str(nb)] = {"strings": k, "ms_median": round(ts[len(ts) // 2] * 1e3, 3), "ms_min": round(ts[0] * 1e3, 3),
                              "mb_s_median": round(nb / ts[len(ts) // 2] / 1e6, 1)}
        small["note"] = ("sw_encode_device on a prefix of the batch, the same handle after the timed launches, "
                         "host clock around each call + device synchronise; median of %d calls" % args.small_steps)

    # PCIe-inclusive rate (rank 0, N=1): the same batch from host buffers to host buffers through
    # sw_encode_batch (Tokenizer.encode_packed).  Reported beside, never `value`.  Two modes: the
    # caller's arrays pinned once (Tokenizer.pin_host: the input read over PCIe by the copy kernel,
    # the ids and offsets written by the device into the caller's arrays) -- `mb_s`; and plain
    # pageable arrays (staged through the library's pinned buffers by host threads) -- `mb_s_pageable`
    e2e = None
    if rank == 0 and world == 1 and args.e2e_steps > 0:
        # the caller's output arrays, allocated and touched once (encode_packed(out=...)): a call then
        # writes the ids into resident pages instead of faulting in a fresh 1 GB array
        out_e = np.zeros(n_bytes, dtype=np.int32)
        oo_e = np.zeros(n_str + 1, dtype=np.int64)
        tok.encode_packed(buf, off, bits, specials=specials, out=out_e, out_off=oo_e)  # (workspace grown once)

        def timed(n):
            dt = 0.0
            for _ in range(n):  # each call timed entry to return
                te = time.perf_counter()
                tok.encode_packed(buf, off, bits, specials=specials, out=out_e, out_off=oo_e)
                dt += time.perf_counter() - te
            return dt / n

        dte_pg = timed(args.e2e_steps)
        st_pg = tok.last_stats
        ids_pg, oo_pg = out_e[:int(oo_e[-1])].copy(), oo_e.copy()
        te = time.perf_counter()  # (one call into a fresh array, for comparison with earlier rounds)
        f_ids, f_off = tok.encode_packed(buf, off, bits, specials=specials)
        dfresh = time.perf_counter() - te
        del f_ids, f_off
        out_e[:] = -1
        pin_modes = {}
        for mode, arrs in (("input", (buf,)), ("all", (buf, out_e, oo_e))):
            tp = time.perf_counter()
            for arr in arrs:
                tok.pin_host(arr)
            t_pin = time.perf_counter() - tp
            tok.encode_packed(buf, off, bits, specials=specials, out=out_e, out_off=oo_e)  # (the direct path's first call)
            dt = timed(args.e2e_steps)
            pin_modes[mode] = (dt, tok.last_stats, t_pin,
                               bool(np.array_equal(oo_e, oo_pg) and np.array_equal(out_e[:len(ids_pg)], ids_pg)))
            for arr in arrs:
                tok.unpin_host(arr)
        best = min(pin_modes, key=lambda m: pin_modes[m][0])
        dte, st, t_pin, same = pin_modes[best]
        same = same and all(v[3] for v in pin_modes.values())
        if dte_pg < dte:  # (which way is faster differs from box to box: the faster one is the line's mb_s)
            best, dte, st = "pageable", dte_pg, st_pg
        e2e = {"mb_s": round(n_bytes / dte / 1e6, 1), "ms": round(dte * 1e3, 2), "ms_h2d": round(st.ms_h2d, 2),
               "ms_kernels": round(st.ms_kernels, 2), "ms_d2h": round(st.ms_d2h, 2),
               "same_token_count": int(oo_e[-1]) == n_tok, "same_ids_pinned_vs_pageable": same,
               "steps": args.e2e_steps,
               "host_buffers": ("pageable numpy in (staged by the library's host threads into its pinned buffers), "
                                "caller-provided resident numpy out (encode_packed out=/out_off=)"
                                if best == "pageable" else
                                "caller's input array pinned once (Tokenizer.pin_host -> sw_encoder_pin_host: read "
                                "over PCIe by the copy kernel, no staging copy); ids as 16 bits through the library's "
                                "pinned buffers, widened into the caller's resident int32 array"
                                if best == "input" else
                                "caller's input and output arrays pinned once (Tokenizer.pin_host -> "
                                "sw_encoder_pin_host: input read over PCIe by the copy kernel, int32 ids and offsets "
                                "written by the device into the caller's arrays)") + ", sw_encode_batch%s" % (
                                   ("_ex (specials found on the host threads: the caller's bitmap)" if host_ps else
                                    "_ex (specials found on the device launch by launch, sw_find_specials_device)")
                                   if specials else ""),
               "mode": best,
               "pinned_modes_mb_s": {m: round(n_bytes / v[0] / 1e6, 1) for m, v in pin_modes.items()},
               "pin_ms_once": round(t_pin * 1e3, 1),
               "pcie_copies": "dma" if args.pipe_dma else "kernels",
               "timing": "mean over calls, each from entry to return",
               "mb_s_pageable": round(n_bytes / dte_pg / 1e6, 1), "ms_pageable": round(dte_pg * 1e3, 2),
               "pageable_ms_h2d_d2h": [round(st_pg.ms_h2d, 2), round(st_pg.ms_d2h, 2)],
               "pageable_note": "pageable numpy in, caller-provided resident numpy out (encode_packed out=/out_off=)",
               "mb_s_fresh_output": round(n_bytes / dfresh / 1e6, 1),
               "fresh_output_note": "pageable, one call with the output array allocated inside it (page faults included)"}
        del out_e, oo_e, ids_pg, oo_pg

    # parity spot-check + CPU baseline (rank 0, N=1 only): the oracle on a bounded prefix of the
    # same corpus; the GPU ids for that prefix must be bit-identical
    cpu = None
    parity = None
    c1 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # configs[0] (C1): 10 MB synthetic ASCII, the reference-trained 500-merge toy model, CPU only
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        t1buf, t1off = corpus.synth(7, corpus.ASCII, 20000, 500, n_threads=args.threads)
        k1 = int(np.searchsorted(t1off, 10_000_000, side="right")) - 1
        t1buf, t1off = t1buf[:int(t1off[k1])], t1off[:k1 + 1]
        toy = Tokenizer(device=local)
        toy.load(os.path.join(ROOT, "tests", "golden", "toy500.model"))
        om1 = oracle.OracleModel(toy.merges)
        tc = time.perf_counter()
        e1 = om1.encode_batch(t1buf, t1off, 0, n_threads=1)
        c1_1 = len(t1buf) / (time.perf_counter() - tc) / 1e6
        tc = time.perf_counter()
        om1.encode_batch(t1buf, t1off, 0, n_threads=args.threads)
        c1_all = len(t1buf) / (time.perf_counter() - tc) / 1e6
        g1 = toy.encode_packed(t1buf, t1off)
        c1 = {"workload": "C1: configs[0], %.1f MB synthetic ASCII, toy500 (reference-trained 500 merges)" % (
                  len(t1buf) / 1e6),
              "cpu_mb_s_1thread": round(c1_1, 3), "cpu_mb_s_all_cores": round(c1_all, 3), "cores": args.threads,
              "kind": "port (oracle/sw_oracle.c)", "python_reference_mb_s": 0.41,
              "gpu_same_ids": bool(np.array_equal(g1[0], e1[0]) and np.array_equal(g1[1], e1[1]))}
        toy.close()
        k = int(np.searchsorted(off, args.cpu_sample_mb * 1e6, side="right")) - 1
        k = max(1, min(k, n_str))
        sbuf, soff = buf[:int(off[k])], off[:k + 1]
        om = oracle.OracleModel(tok.merges)
        def cpu_encode(nt):
            if specials:
                return om.encode_batch_specials(sbuf, soff, specials, pat, n_threads=nt)
            return om.encode_batch(sbuf, soff, pat, n_threads=nt)
        tc = time.perf_counter()
        ids_cpu, ooff_cpu = cpu_encode(1)
        dt1 = time.perf_counter() - tc
        tc = time.perf_counter()
        cpu_encode(args.threads)
        dtm = time.perf_counter() - tc
        got = d_out[:int(ooff_cpu[-1])].cpu().numpy()
        if out16:
            got = got.astype(np.int32) & 0xFFFF
        got_off = d_oo[:k + 1].cpu().numpy()
        parity = bool(np.array_equal(got, ids_cpu) and np.array_equal(got_off, ooff_cpu))
        cpu = {"value": round(len(sbuf) / dt1 / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
               "sample": "first %d strings (%.1f MB) of the same corpus, oracle/sw_oracle.c, 1 thread, "
                         "host pre-split + merge loop" % (k, len(sbuf) / 1e6),
               "value_all_cores": round(len(sbuf) / dtm / 1e6, 3), "cores_all": args.threads,
               "usable_cores": usable_cores, "machine_cpus": machine_cpus, "cpu_model": cpu_model,
               "c1": c1, "python_reference_mb_s": 0.33}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": ("C5 stress, 50k merges" if c5 else
                                    ("C3: configs[2], host %s pre-split%s, GPU merge loop" % (
                                        args.pattern, " + special tokens on host" if specials else "")) if host_ps else
                                    ("C2: configs[1] full path, 1 GiB %s UTF-8, %d strings, GPU %s pre-split + "
                                     "merge loop + id compaction%s" % (
                                         (args.corpus or "mixed").upper(), n_str, args.pattern,
                                         (" + special tokens (found on the device, inside the step)" if sp_device
                                          else " + special tokens (found on host)") if specials else "")))
                       + (" + RCCL all-gather of ids + reassembly (offsets rebased, ids widened to int32)"
                          if gather else ""),
                       "presplit": args.presplit,
                       "bytes_per_rank": n_bytes, "strings_per_rank": n_str, "merges": len(tok.merges),
                       "model": model, "pattern": args.pattern, "parallelism": "doc-shard x%d" % world,
                       "corpus": corpus_name,
                       "gather_in_step": gather, "gather_overlaps_next_encode": overlap, "gather_id_bits": id_bits if gather else None,
                       "encode_out_bits": 16 if out16 else 32,
                       "chunk_table": not args.no_chunk_table,
                       "dedupe": not args.no_dedupe},
            "mtok_per_s": round(all_tok * args.steps / sec / 1e6, 3),
            "bytes_per_token": round(all_bytes / max(all_tok, 1), 4),
            "chunks": int(all_chunks),
            "rates": rates,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity_vs_oracle_sample": parity,
            "reassembly_check": reassembly_ok,
            "e2e_pcie": e2e,
            "small_batches": small,
            "host_prep_s": round(t_prep, 2),
            "host_split_s": round(t_split, 3) if (host_ps or specials) else None,
            "host_split_note": ("host threads, outside the timed GPU step: special-token occurrences%s (%d threads)" % (
                " + %s pre-split bitmap" % args.pattern if host_ps else "", args.threads)) if (host_ps or specials) else None,
            "specials": ({"per_kib": args.specials, "occurrences": int(len(sp_host[0])), "tokens": SPECIALS,
                          "end_of_string": "<|endoftext|>", "found": "device" if sp_device else "host",
                          "found_note": ("sw_find_specials_device inside the timed step (its kernels before the "
                                         "encode's; roofline.kernel_ms = the whole step)" if sp_device else
                                         "host threads, before the timed step (host_split_s)"),
                          "device_count_equals_host": sp_dev_ok} if specials else None),
        }
        print(json.dumps(line), flush=True)
    tok.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
