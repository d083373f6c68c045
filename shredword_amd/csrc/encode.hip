// MI355X (gfx950) batched BPE encode: kernels + host orchestration + the C-ABI.
//
// Semantics (exact, for ANY merge table): per pre-split chunk, ids = chunk bytes; while at
// least two ids remain, find the adjacent pair with the lowest merges-value (first occurrence
// wins ties), stop if no pair is in merges, else replace every non-overlapping occurrence of
// that pair, left to right, by the value.  This is the loop the reference's primitives
// compose: get_stats (shredword/base.py:10-20), min over merges.get (base.py:107-108 leaves
// encode abstract), merge (base.py:22-36).
//
// Device pipeline (all on one stream; inputs resident in HBM; kernels in kernels.h):
//   k_tile_strings   first string of each tile
//   k_classify       per 2 KiB tile: single bytes + whole-chunk-table hits settled, one slot
//                    per chunk, repeats of a multi-token chunk deduped, the rest queued by
//                    length bucket
//   k_scan_*/k_scatter  dense bucket-major merge queue
//   k_merge_bucket   exact merge loop of the distinct queued chunks, one chunk per lane, in
//                    registers (N = 4/8/16/32)
//   k_merge_long     wave-cooperative merge loop for chunks > 32 bytes
//   k_tile_count     ids per tile, then k_scan_* for the tile bases
//   k_compact        slots -> contiguous ids; string chunk index -> id offset
//   k_string_offsets final per-string offsets
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "capi.h"
#include "hostpool.h"
#include "kernels.h"
#include "long_split.h"
#include "presplit_kernel.h"
#include "split_classify.h"
#include "copy_seg.h"
#include "specials_find.h"
#include "shredword_hip.h"
#include "test_options.h"
#include "table.h"

using namespace sw;

// ------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------
static thread_local std::string g_err;
int32_t sw::set_error(int32_t code, const std::string& msg) {
  g_err = msg;
  return code;
}
static int32_t fail(int32_t code, const std::string& msg) { return sw::set_error(code, msg); }
#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(SW_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

extern "C" const char* sw_last_error(void) { return g_err.c_str(); }
extern "C" const char* sw_version(void) { return "shredword_hip 0.1 gfx950"; }
extern "C" int32_t sw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct sw_encoder {
  int device = 0;
  hipStream_t stream = nullptr;
  DevTable table{};
  void* d_table = nullptr;
  int64_t n_merges = 0;
  bool ids16 = false;  // every pair member and value <= 0xFFFD: 16-bit ids in the kernels
  DevChunkTable chunks{};
  void* d_chunks = nullptr;
  int64_t n_chunk_entries = 0;
  int64_t chunk_table_bytes = 0;
  // split + verify for long chunks (long_split.h): well-formed tables only
  bool split_ok = false;              // values >= 256, unique, larger than both pair members
  bool long_split = true;             // SW_OPT_LONG_SPLIT (0: the wave loop per long chunk)
  uint2* d_inv = nullptr;             // merge value -> pair
  uint32_t n_inv = 0;
  int64_t max_launch = kMaxLaunchBytes;  // SW_OPT_MAX_LAUNCH_BYTES (sw_encode_batch splits above it)
  int n_cu = 256;                     // compute units (persistent grids)
  // the workspace is reused by every call: a call on another stream waits for the last one
  hipEvent_t ws_done = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_pending = false;
  int64_t last_tiles = 0;             // tiles of the last sw_encode_device launch (sw_encoder_last_counts)
  // sw_encode_batch's pipeline for large host batches (SW_OPT_PIPE_RUN_BYTES): runs of whole
  // strings go host -> pinned -> device -> encode -> (16-bit ids when they fit) -> pinned -> host,
  // run k's copies overlapping run k-1's encode; two slots of buffers
  struct Pinned {                     // sw_encoder_pin_host: a caller's range and its device address
    char* h = nullptr;
    int64_t n = 0;
    char* d = nullptr;
  };
  std::vector<Pinned> pins;
  int64_t* d_done = nullptr;          // the direct push (pinned caller arrays): ids written so far, overflow flag
  // (device address of [p, p + n) when it lies in a pinned range, else nullptr)
  void* pinned_dev(const void* p, int64_t n) const {
    for (const Pinned& r : pins)
      if ((const char*)p >= r.h && (const char*)p + n <= r.h + r.n) return r.d + ((const char*)p - r.h);
    return nullptr;
  }
  struct PipeSlot {
    uint8_t* h_in = nullptr; int64_t* h_off = nullptr; uint64_t* h_bits = nullptr;  // pinned
    void* h_out = nullptr; int64_t* h_oo = nullptr; int64_t* h_ntok = nullptr;        // pinned
    uint8_t* d_in = nullptr; int64_t* d_off = nullptr; uint64_t* d_bits = nullptr;
    int32_t* d_out = nullptr; int64_t* d_oo = nullptr; uint16_t* d_out16 = nullptr;
    int64_t* d_ntok = nullptr;  // this run's token count, kept apart from the shared workspace
    int64_t* h_sp = nullptr; int64_t* d_sp = nullptr;  // special-token occurrences: pos | len, id (3 x cap_sp x 8 B)
    int64_t cap_sp = 0;
    hipEvent_t e_in = nullptr, e_comp = nullptr, e_out = nullptr;
    int64_t cap_bytes = 0, cap_str = 0;
  } pipe[4];
  int pipe_depth = 3;                 // SW_OPT_PIPE_DEPTH: runs in flight (slots)
  int64_t pipe_run = 128LL << 20;     // run size; batches over 2 runs take the pipeline (0: never; 128 MiB: e2e
                                      // 28.2 -> 30.1 GB/s pageable, 29.9 -> 31.8 pinned input against 64 MiB, r4z)
  bool pipe_kcopy = true;             // SW_OPT_PIPE_COPY_KERNELS
  hipStream_t s_h2d = nullptr, s_d2h = nullptr;
  // the merge kernels of different length buckets are independent: forked onto these streams
  // they overlap (each alone leaves most of the chip idle), joined before k_tile_count
  bool merge_fork = true;             // SW_OPT_MERGE_STREAMS
  hipStream_t s_fork[2] = {nullptr, nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
  hipEvent_t ev_fork_long = nullptr;  // (the long chunks' fork, right after k_classify)
  sw::HostPool* pool = nullptr;
  // workspace
  int64_t cap_bytes = -1, cap_str = -1;
  int32_t* d_scratch = nullptr;
  uint32_t* d_res = nullptr;          // [2 * n_bytes] merge results, double-spaced position space
  int64_t* d_part = nullptr;
  int64_t* d_tile_slo = nullptr;
  int64_t* d_tile_sp = nullptr;       // first special-token occurrence at or after each tile
  uint32_t* d_tile_slots = nullptr;
  uint32_t* d_tile_nref = nullptr;
  uint32_t* d_rlist = nullptr;
  uint64_t* d_queue = nullptr;        // dense merge queue (bucket-major)
  uint32_t* d_bcnt = nullptr;         // [kNumBuckets * n_tiles] queued chunks per (bucket, tile)
  int64_t* d_boff = nullptr;          // its exclusive scan
  int64_t* d_qtotal = nullptr;
  unsigned long long* d_stamps = nullptr;  // SW_STAMPS builds
  uint64_t* d_dtab = nullptr;         // chunk dedupe table
  uint32_t dmask = 0;
  int64_t dd_slots = 0;               // entries of d_dtab (grown by grow_dedupe, kept across workspace reallocations)
  unsigned long long* d_ddfull = nullptr;     // per launch: dedupable chunks that found every candidate taken
  unsigned long long* h_ddfull = nullptr;     // ... published by k_string_offsets (host-mapped, coherent)
  unsigned long long* hd_ddfull = nullptr;    // (its device address)
  uint4* d_dres = nullptr;            // dense result heads, one per table entry
  uint8_t* d_dcnt = nullptr;          // their id counts (<= 32), one byte per table entry
  uint32_t* d_big = nullptr;          // chunks over kLongLds bytes: count, then their long-list indices
  // long chunks by split + verify (long_split.h): per long chunk, per piece, piece ids, counters
  void* d_lp = nullptr;               // one allocation, carved into LongArgs
  LongArgs lp{};
  int64_t* d_lpart = nullptr;         // scan partials for the piece / chunk scans
  bool dedupe = true;
  bool dedupe_exact = true;           // SW_OPT_DEDUPE_EXACT
  int64_t dedupe_slots = 0;           // SW_OPT_DEDUPE_SLOTS (0: automatic)
  bool dd_grow_stop = false;          // a growth allocation failed: keep the table that works
  int32_t test_fail_grow = 0;         // SW_OPT_TEST_FAIL_GROWTH: the next growth's allocations fail (tests)
  int32_t pattern = SW_PAT_CL100K;    // SW_OPT_PATTERN: device pre-split of sw_encode_device(bits = NULL)
  bool host_presplit = false;         // SW_OPT_HOST_PRESPLIT: sw_encode_batch pre-splits on the host
  uint64_t* d_pbits = nullptr;        // [n_bytes / 64] device pre-split bitmap
  uint32_t* d_edge = nullptr;         // [kEdgeWords][n_tiles + 1] k_edges: the tile boundaries' masks and words
  unsigned int* d_redo = nullptr;     // k_split_classify's tiles for k_split_redo: count, then the list (int64)
  bool fused_presplit = true;         // SW_OPT_FUSED_PRESPLIT: the device pre-split inside k_split_classify
  bool device_specials = true;        // SW_OPT_DEVICE_SPECIALS: sw_encode_batch_ex finds specials on the device
  int compact_kernel = 0;
  int staged_heads = 0;               // SW_OPT_STAGED_HEADS: 0 automatic (a grown dedupe table), 1 always, 2 never  // SW_OPT_COMPACT_KERNEL (0: from the last launch's ids per tile)
  int64_t cp_prev_tiles = 0;          // tiles of the previous launch (its id count: h_ddfull[1])
  unsigned long long* d_pcount = nullptr;
  uint64_t* d_llist = nullptr;        // k_classify's long chunks (EncArgs::llist) and their count
  unsigned long long* d_lcount = nullptr;
  uint32_t dedupe_fp_mask = (1u << 26) - 1;
  uint32_t* d_tile_cnt = nullptr;
  int64_t* d_tile_base = nullptr;
  int64_t* d_total = nullptr;
  // host-path staging
  int64_t io_bytes = -1, io_str = -1;
  uint8_t* d_bytes = nullptr;
  int64_t* d_str_off = nullptr;
  uint64_t* d_bits = nullptr;
  int32_t* d_out = nullptr;
  int64_t* d_out_off = nullptr;
  // the device special-token finder (specials_find.h): the specials' table, keyed by content, and
  // its per-tile work arrays
  void* d_spt = nullptr;
  SpTab spt{};
  std::string spt_key;                // the specials the table holds (bytes, offsets, ids)
  bool spt_dev = false;               // every special fits the device finder (<= kSpMaxLen bytes)
  int32_t spt_min_len = 1;            // the shortest non-empty special
  int64_t spf_tiles = 0;              // capacity of the finder's arrays, in tiles
  int64_t spf_tcap = 0;               // ... and occurrences per tile
  uint32_t* d_spf = nullptr;          // candidate bits, occurrence bits, per-tile counts, flag
  uint32_t* d_spf_list = nullptr;     // per tile, its occurrences (k_sp_find)
  int64_t* d_spf_off = nullptr;       // per-tile occurrence offsets, twice (+ scan partials, totals)
  int64_t* d_nsp = nullptr;           // sw_encode_batch_ex: the finder's count
  int64_t sp_cap = 0;                 // special-token occurrences staged for sw_encode_batch_ex
  int64_t* d_sp_pos = nullptr;
  int32_t* d_sp_len = nullptr;
  int32_t* d_sp_id = nullptr;
  // dominant-kernel timing: one event pair per launch since sw_encoder_set_timing(h, 1)
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;  // pairs recorded
  std::vector<hipEvent_t> ev_cls;  // (timing) the classification kernel of each launch: a pair per launch
  size_t ev_cls_used = 0;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

void free_workspace(sw_encoder* h) {
  (void)hipFree(h->d_scratch); (void)hipFree(h->d_res); (void)hipFree(h->d_pbits); (void)hipFree(h->d_edge); (void)hipFree(h->d_redo); (void)hipFree(h->d_pcount); (void)hipFree(h->d_part);
  (void)hipFree(h->d_ddfull); h->d_ddfull = nullptr;
  (void)hipFree(h->d_llist); h->d_llist = nullptr;
  (void)hipFree(h->d_lcount); h->d_lcount = nullptr;
  (void)hipFree(h->d_tile_slo); (void)hipFree(h->d_tile_sp); (void)hipFree(h->d_stamps);
  (void)hipFree(h->d_tile_slots); (void)hipFree(h->d_tile_nref); (void)hipFree(h->d_rlist); (void)hipFree(h->d_queue); (void)hipFree(h->d_bcnt); (void)hipFree(h->d_boff);
  (void)hipFree(h->d_qtotal);
  h->d_tile_slo = nullptr; h->d_tile_sp = nullptr; h->d_stamps = nullptr; h->d_tile_slots = nullptr; h->d_tile_nref = nullptr; h->d_rlist = nullptr; h->d_queue = nullptr;
  h->d_bcnt = nullptr; h->d_boff = nullptr; h->d_qtotal = nullptr;
  (void)hipFree(h->d_dtab); (void)hipFree(h->d_tile_base); (void)hipFree(h->d_tile_cnt);
  (void)hipFree(h->d_dres); (void)hipFree(h->d_big); (void)hipFree(h->d_dcnt);
  (void)hipFree(h->d_lp); (void)hipFree(h->d_lpart);
  h->d_dres = nullptr; h->d_big = nullptr; h->d_dcnt = nullptr; h->d_lp = nullptr; h->d_lpart = nullptr;
  h->lp = LongArgs{};
  (void)hipFree(h->d_total);
  h->d_scratch = nullptr; h->d_res = nullptr; h->d_pbits = nullptr; h->d_edge = nullptr; h->d_redo = nullptr; h->d_pcount = nullptr; h->d_part = nullptr;
  h->d_dtab = nullptr; h->d_tile_base = nullptr; h->d_tile_cnt = nullptr; h->d_total = nullptr;
  h->cap_bytes = -1; h->cap_str = -1;
}

void free_io(sw_encoder* h) {
  (void)hipFree(h->d_bytes); (void)hipFree(h->d_str_off); (void)hipFree(h->d_bits);
  (void)hipFree(h->d_out); (void)hipFree(h->d_out_off);
  (void)hipFree(h->d_sp_pos); (void)hipFree(h->d_sp_len); (void)hipFree(h->d_sp_id);
  h->d_sp_pos = nullptr; h->d_sp_len = nullptr; h->d_sp_id = nullptr; h->sp_cap = 0;
  h->d_bytes = nullptr; h->d_str_off = nullptr; h->d_bits = nullptr; h->d_out = nullptr; h->d_out_off = nullptr;
  h->io_bytes = -1; h->io_str = -1;
}

void free_pipe(sw_encoder* h) {
  for (auto& p : h->pipe) {
    (void)hipHostFree(p.h_in); (void)hipHostFree(p.h_off); (void)hipHostFree(p.h_bits); (void)hipHostFree(p.h_out);
    (void)hipHostFree(p.h_oo); (void)hipHostFree(p.h_ntok);
    (void)hipFree(p.d_in); (void)hipFree(p.d_off); (void)hipFree(p.d_bits); (void)hipFree(p.d_out); (void)hipFree(p.d_oo);
    (void)hipFree(p.d_out16); (void)hipFree(p.d_ntok);
    (void)hipHostFree(p.h_sp); (void)hipFree(p.d_sp);
    if (p.e_in) (void)hipEventDestroy(p.e_in);
    if (p.e_comp) (void)hipEventDestroy(p.e_comp);
    if (p.e_out) (void)hipEventDestroy(p.e_out);
    p = sw_encoder::PipeSlot{};
  }
}

constexpr unsigned long long kStagedMinMerges = 6000000;  // (see encode_device: k_tile_count_staged)

int32_t ensure_workspace(sw_encoder* h, int64_t n_bytes) {
  if (n_bytes <= h->cap_bytes) return SW_OK;
  free_workspace(h);
  const int64_t nb = std::max<int64_t>(n_bytes, 1);
  const int64_t n_tiles = (nb + kTile - 1) / kTile;
  HIP_TRY(hipMalloc(&h->d_scratch, sizeof(int32_t) * n_tiles * kTile));  // whole tiles: see k_compact
  // (+ slack for k_compact's head reads; k_classify's tile-local queue, aliased here, takes whole tiles)
  HIP_TRY(hipMalloc(&h->d_res, sizeof(uint32_t) * std::max<int64_t>(2 * nb + 16, n_tiles * kTile)));
  HIP_TRY(hipMalloc(&h->d_tile_slo, sizeof(int64_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_tile_sp, sizeof(int64_t) * 2 * (n_tiles + 1)));  // (tile_sp, then tile_spw)
  HIP_TRY(hipMalloc(&h->d_tile_slots, sizeof(uint32_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_tile_nref, sizeof(uint32_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_rlist, sizeof(uint32_t) * n_tiles * kTile));
  // queued chunks have >= 2 bytes: at most nb / 2 of them
  HIP_TRY(hipMalloc(&h->d_queue, sizeof(uint64_t) * (nb / 2 + 64)));
  HIP_TRY(hipMalloc(&h->d_bcnt, sizeof(uint32_t) * kNumBuckets * n_tiles));
  HIP_TRY(hipMalloc(&h->d_boff, sizeof(int64_t) * kNumBuckets * n_tiles));
  HIP_TRY(hipMalloc(&h->d_qtotal, sizeof(int64_t)));
  HIP_TRY(hipMalloc(&h->d_part, sizeof(int64_t) * ((kNumBuckets * n_tiles + kScanBlock - 1) / kScanBlock + 1)));
  {  // dedupe table: ~1 entry per 64 input bytes, 2^6 .. 2^22 entries (64 MiB) to start with, more
     // when a launch overflows it (grow_dedupe), and a 16-byte result head + a count byte per entry
    int64_t slots = 64;
    while (slots < nb / 64 && slots < kDdSlotsDefault) slots <<= 1;
    slots = std::max(slots, h->dd_slots);
    h->dd_slots = slots;
    HIP_TRY(hipMalloc(&h->d_dtab, sizeof(uint64_t) * kDdWords * (slots)));
    HIP_TRY(hipMalloc(&h->d_dres, sizeof(uint4) * (slots)));
    HIP_TRY(hipMalloc(&h->d_dcnt, slots));
    h->dmask = (uint32_t)(slots - 1);
  }
  HIP_TRY(hipMalloc(&h->d_big, sizeof(uint32_t) * (nb / (kLongLds + 1) + 2)));  // (count + list)
  {  // long_split.h: a long chunk has > kShort bytes and ceil(len / kPieceW) pieces
    const int64_t lcap = nb / (kShort + 1) + 64, pcap = nb / kPieceW + lcap;  // (ceil(len / W) pieces a chunk)
    const size_t bytes = 8 * (size_t)kLcAlloc + 4 * (size_t)lcap * 7 + 8 * (size_t)lcap  // chunks
                         + 4 * (size_t)pcap * 11                                         // pieces, lists
                         + 4 * (size_t)(nb + 64) + 4 * (size_t)pcap + 1024;             // ids, window list (+ alignment)
    HIP_TRY(hipMalloc(&h->d_lp, bytes));
    char* q = (char*)h->d_lp;
    auto take = [&](size_t n) { char* r = q; q += (n + 15) & ~(size_t)15; return (void*)r; };
    LongArgs& L = h->lp;
    L.ctl = (int64_t*)take(8 * (size_t)kLcAlloc);
    L.lpo = (int64_t*)take(8 * (size_t)lcap);
    L.lstart = (uint32_t*)take(4 * (size_t)lcap); L.llen = (uint32_t*)take(4 * (size_t)lcap);
    L.lnp = (uint32_t*)take(4 * (size_t)lcap); L.lfall = (uint32_t*)take(4 * (size_t)lcap);
    L.flist = (uint32_t*)take(4 * (size_t)lcap);
    L.wstart = (uint32_t*)take(4 * (size_t)lcap); L.wlen = (uint32_t*)take(4 * (size_t)lcap);
    L.pbeg = (uint32_t*)take(4 * (size_t)pcap); L.pcnt = (uint32_t*)take(4 * (size_t)pcap);
    L.pchunk = (uint32_t*)take(4 * (size_t)pcap); L.pflag = (uint32_t*)take(4 * (size_t)pcap);
    L.pprev = (uint32_t*)take(4 * (size_t)pcap); L.pnext = (uint32_t*)take(4 * (size_t)pcap);
    L.jlist[0] = (uint32_t*)take(4 * (size_t)pcap); L.jlist[1] = (uint32_t*)take(4 * (size_t)pcap);
    L.clist = (uint32_t*)take(4 * (size_t)pcap); L.hlist = (uint32_t*)take(4 * (size_t)pcap);
    L.pseen = (uint32_t*)take(4 * (size_t)pcap);
    L.pid = (uint32_t*)take(4 * (size_t)(nb + 64));
    L.wlist = (uint32_t*)take(4 * (size_t)pcap);
    L.lcap = lcap;
    L.pcap = pcap;
    HIP_TRY(hipMalloc(&h->d_lpart, sizeof(int64_t) * kDscanGrid));
  }
  HIP_TRY(hipMalloc(&h->d_tile_base, sizeof(int64_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_tile_cnt, sizeof(uint32_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_total, sizeof(int64_t)));
  HIP_TRY(hipMalloc(&h->d_pbits, sizeof(uint64_t) * ((nb + 63) / 64)));
  HIP_TRY(hipMalloc(&h->d_edge, sizeof(uint32_t) * kEdgeWords * (n_tiles + 1)));
  HIP_TRY(hipMalloc(&h->d_redo, sizeof(int64_t) * (n_tiles + 1)));
  HIP_TRY(hipMalloc(&h->d_pcount, sizeof(unsigned long long)));
  HIP_TRY(hipMalloc(&h->d_ddfull, sizeof(unsigned long long)));
  HIP_TRY(hipMalloc(&h->d_llist, sizeof(uint64_t) * (nb / (kShort + 1) + 64)));
  HIP_TRY(hipMalloc(&h->d_lcount, sizeof(unsigned long long)));
  HIP_TRY(hipMemset(h->d_ddfull, 0, sizeof(unsigned long long)));
#ifdef SW_STAMPS
  HIP_TRY(hipMalloc(&h->d_stamps, sizeof(unsigned long long) * 32 * 64));  // 64 copies per counter
  HIP_TRY(hipMemset(h->d_stamps, 0, sizeof(unsigned long long) * 32 * 64));
#endif
  h->cap_bytes = nb;
  return SW_OK;
}

// Two-choice cuckoo table (see table.h).  Narrow buckets hold 2 slots, wide buckets 1; the
// bucket count starts at the load factor below and doubles (with fresh hash multipliers) until
// every pair is placed.
// the quotient table (table.h) for 16-bit ids: buckets = the smallest power of two >= 2^16 with at
// most SW_Q16_FILL keys per bucket on average; constants redrawn (eight tries per size, then the
// buckets double) until no bucket holds more than four keys
bool build_q16(const std::unordered_map<uint64_t, int32_t>& dict, const std::vector<uint64_t>& order, DevTable* t,
               std::vector<uint4>* out) {
  uint32_t log2b = 16;
  while ((double)(1ull << log2b) * 0.25 < (double)order.size()) ++log2b;
  uint64_t rng = 0x452821E638D01377ULL;
  auto next = [&]() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; };
  for (int attempt = 0; attempt < 64 && log2b <= 24; ++attempt) {
    if (attempt && attempt % 8 == 0) ++log2b;
    const size_t nb = (size_t)1 << log2b;
    t->shift = 32 - log2b;
    t->m1 = (uint32_t)next() | 1u;
    t->m2 = (uint32_t)next() | 1u;
    std::vector<uint32_t> w(nb * 4, 0xFFFFFFFFu);
    std::vector<uint8_t> fill(nb, 0);
    bool ok = true;
    for (uint64_t k : order) {
      const uint32_t a = (uint32_t)(k >> 32), c = (uint32_t)k, v = (uint32_t)dict.at(k);
      const uint32_t x = q16_mix((a << 16) | c, t->m1, t->m2);
      const uint32_t bk = x >> t->shift;
      if (fill[bk] == 4) { ok = false; break; }
      w[4 * (size_t)bk + fill[bk]++] = (x & 0xFFFFu) | (v << 16);
    }
    if (!ok) continue;
    out->assign(nb, make_uint4(0, 0, 0, 0));
    std::memcpy(out->data(), w.data(), w.size() * sizeof(uint32_t));
    t->q16 = 1;
    return true;
  }
  return false;
}

bool build_cuckoo(const std::unordered_map<uint64_t, int32_t>& dict, const std::vector<uint64_t>& order, bool wide,
                  DevTable* t, std::vector<uint4>* out) {
  const int slots = wide ? 1 : 2;
  const double max_load = wide ? 0.40 : 0.80;
  uint32_t log2b = 4;
  while ((double)(1ull << log2b) * slots * max_load < (double)order.size()) ++log2b;
  uint64_t rng = 0x243F6A8885A308D3ULL;
  auto next = [&]() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; };
  for (int attempt = 0; attempt < 64; ++attempt) {
    if (attempt && attempt % 4 == 0 && log2b < 30) ++log2b;
    const size_t nb = (size_t)1 << log2b;
    t->shift = 32 - log2b;
    t->m1 = (uint32_t)next() | 1u;
    t->m2 = (uint32_t)next() | 1u;
    std::vector<uint4> b(nb, make_uint4(kEmptyKey, 0, kEmptyKey, 0));
    bool ok = true;
    for (uint64_t k : order) {
      uint32_t a = (uint32_t)(k >> 32), c = (uint32_t)k, v = (uint32_t)dict.at(k);
      for (int kick = 0;; ++kick) {
        if (kick > 500) { ok = false; break; }
        const uint32_t f = mix_key(a, c);
        const uint32_t c1 = bucket1(f, *t), c2 = bucket2(f, *t);
        bool placed = false;
        for (uint32_t bk : {c1, c2}) {
          uint4& q = b[bk];
          if (wide) {
            if (q.x == kEmptyKey) { q = make_uint4(a, c, v, 0); placed = true; break; }
          } else {
            const uint32_t key = (a << 16) | c;
            if (q.x == kEmptyKey) { q.x = key; q.y = v; placed = true; break; }
            if (q.z == kEmptyKey) { q.z = key; q.w = v; placed = true; break; }
          }
        }
        if (placed) break;
        // evict a random resident of a random candidate bucket and re-insert it
        uint4& q = b[(next() & 1) ? c1 : c2];
        if (wide) {
          uint4 old = q;
          q = make_uint4(a, c, v, 0);
          a = old.x; c = old.y; v = old.z;
        } else {
          const uint32_t key = (a << 16) | c;
          uint32_t ok_, ov;
          if (next() & 1) { ok_ = q.x; ov = q.y; q.x = key; q.y = v; }
          else { ok_ = q.z; ov = q.w; q.z = key; q.w = v; }
          a = ok_ >> 16; c = ok_ & 0xFFFF; v = ov;
        }
      }
      if (!ok) break;
    }
    if (ok) { out->swap(b); return true; }
  }
  return false;
}


// device pre-split of [d_bytes, d_bytes + n_bytes) into d_bits (every dword of the bitmap is
// stored: no clearing)
hipError_t launch_presplit(hipStream_t st, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                           int64_t n_str, int32_t pattern, uint64_t* d_bits, const int64_t* d_tile_slo) {
  if (n_bytes <= 0) return hipSuccess;
  PbArgs g{d_bytes, n_bytes, d_str_off, n_str, d_tile_slo};
  hipLaunchKernelGGL(k_presplit_bits, dim3((unsigned)((n_bytes + kPbBlock - 1) / kPbBlock)), dim3(kPbThreads), 0, st, g,
                     (int)pattern, (uint32_t*)d_bits);
  return hipGetLastError();
}

}  // namespace

// exclusive scan of cnt[0..n) into base, total into *total (two small kernels: the blocks' sums,
// then each block's scan behind the sum of the sums before it)
hipError_t sw::launch_scan(hipStream_t st, const uint32_t* cnt, int64_t n, int64_t* part, int64_t* base,
                           int64_t* total, const int64_t* n_dev) {
  const int64_t n_parts = (n + kScanBlock - 1) / kScanBlock;
  if (n_parts == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(int64_t), st);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)n_parts), dim3(kThreads), 0, st, cnt, n, n_dev, part);
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)n_parts), dim3(kThreads), 0, st, cnt, n, n_dev, part, base, total);
  return hipGetLastError();
}
int64_t sw::scan_block() { return kScanBlock; }

extern "C" int32_t sw_encoder_create(const int32_t* pairs, const int32_t* vals, int64_t n, int32_t device,
                                     sw_encoder** out) {
  if (!out || n < 0 || (n > 0 && (!pairs || !vals))) return fail(SW_ERR_ARG, "sw_encoder_create: bad arguments");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(SW_ERR_NODEV, "sw_encoder_create: no HIP device visible");
  if (device < 0 || device >= ndev) return fail(SW_ERR_ARG, "sw_encoder_create: bad device ordinal");
  // dict semantics: the last value of a duplicated pair wins (base.py:145-148)
  std::unordered_map<uint64_t, int32_t> dict;
  dict.reserve((size_t)n * 2);
  std::vector<uint64_t> order;
  order.reserve((size_t)n);
  bool wide = false, ids16 = true;
  for (int64_t i = 0; i < n; ++i) {
    int32_t a = pairs[2 * i], b = pairs[2 * i + 1], v = vals[i];
    if (a < 0 || b < 0) return fail(SW_ERR_ARG, "sw_encoder_create: negative token id in a pair");
    if (v < 0) return fail(SW_ERR_ARG, "sw_encoder_create: negative merge value");
    uint64_t k = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
    auto it = dict.find(k);
    if (it == dict.end()) { dict.emplace(k, v); order.push_back(k); }
    else it->second = v;
    if (a > 0xFFFF || b > 0xFFFF || (a == 0xFFFF && b == 0xFFFF)) wide = true;
    if (a > 0xFFFD || b > 0xFFFD || v > 0xFFFD) ids16 = false;
  }
  // well-formed (the split path's precondition, kernels.h): every value >= 256, unique, and
  // larger than both members of its pair
  bool split_ok = true;
  uint32_t max_v = 0;
  {
    std::unordered_set<int32_t> vals;
    vals.reserve(order.size() * 2);
    for (uint64_t k : order) {
      const int32_t v = dict.at(k), a = (int32_t)(k >> 32), b = (int32_t)(uint32_t)k;
      if (v < 256 || v <= a || v <= b || !vals.insert(v).second) split_ok = false;
      max_v = std::max<uint32_t>(max_v, (uint32_t)v);
    }
    if (max_v >= (1u << 26)) split_ok = false;  // (inverse table bounded to 512 MiB)
  }
  sw_encoder* h = new sw_encoder();
  h->device = device;
  h->n_merges = (int64_t)order.size();
  h->split_ok = split_ok && !order.empty();
  h->table.wide = wide ? 1u : 0u;
  h->ids16 = ids16 && !wide;
  std::vector<uint4> host;
  h->table.q16 = 0;
  if (!(ids16 && !wide && build_q16(dict, order, &h->table, &host)) && !build_cuckoo(dict, order, wide, &h->table, &host)) {
    delete h;
    return fail(SW_ERR_ALLOC, "sw_encoder_create: could not build the pair table");
  }
  const size_t table_bytes = host.size() * sizeof(uint4);
  ChunkTableHost ct;
  if (!build_chunk_table(dict, order, &ct)) {
    delete h;
    return fail(SW_ERR_ALLOC, "sw_encoder_create: could not build the chunk table");
  }
  h->n_chunk_entries = (int64_t)(ct.n_short + ct.n_long);
  DeviceGuard g(device);
  {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0) h->n_cu = cu;
  }
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&h->d_table, table_bytes);
  if (e == hipSuccess) e = hipMemcpy(h->d_table, host.data(), table_bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    sw_encoder_destroy(h);
    return fail(SW_ERR_HIP, std::string("sw_encoder_create: ") + hipGetErrorString(e));
  }
  h->table.buckets = h->d_table;
  {
    const size_t sb = ct.sb.size() * sizeof(uint4), lb = ct.lb.size() * sizeof(uint4);
    e = hipMalloc(&h->d_chunks, sb + lb);
    if (e == hipSuccess) e = hipMemcpy(h->d_chunks, ct.sb.data(), sb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy((char*)h->d_chunks + sb, ct.lb.data(), lb, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      sw_encoder_destroy(h);
      return fail(SW_ERR_HIP, std::string("sw_encoder_create: ") + hipGetErrorString(e));
    }
    h->chunk_table_bytes = (int64_t)(sb + lb);
    h->chunks.sb = (const uint4*)h->d_chunks;
    h->chunks.lb = (const uint4*)((char*)h->d_chunks + sb);
    h->chunks.s_shift = ct.s_shift; h->chunks.s_m1 = ct.s_m1; h->chunks.s_m2 = ct.s_m2;
    h->chunks.l_shift = ct.l_shift; h->chunks.l_m1 = ct.l_m1; h->chunks.l_m2 = ct.l_m2;
    h->chunks.enabled = 1;
  }
  if (h->split_ok) {
    std::vector<uint2> inv((size_t)max_v + 1, make_uint2(kInf, kInf));
    for (uint64_t k : order) inv[(size_t)dict.at(k)] = make_uint2((uint32_t)(k >> 32), (uint32_t)k);
    e = hipMalloc(&h->d_inv, inv.size() * sizeof(uint2));
    if (e == hipSuccess) e = hipMemcpy(h->d_inv, inv.data(), inv.size() * sizeof(uint2), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      sw_encoder_destroy(h);
      return fail(SW_ERR_HIP, std::string("sw_encoder_create: ") + hipGetErrorString(e));
    }
    h->n_inv = (uint32_t)inv.size();
  }
  e = hipEventCreateWithFlags(&h->ws_done, hipEventDisableTiming);
  if (e == hipSuccess)  // (the dedupe overflow count of the last launch, written by the device)
    e = hipHostMalloc((void**)&h->h_ddfull, 3 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    h->h_ddfull[0] = 0;  // (and [1]: the last launch's id count)
    h->h_ddfull[1] = 0;
    h->h_ddfull[2] = 0;  // (and [2]: its merge loops)
    e = hipHostGetDevicePointer((void**)&h->hd_ddfull, h->h_ddfull, 0);
  }
  if (e != hipSuccess) {
    sw_encoder_destroy(h);
    return fail(SW_ERR_HIP, std::string("sw_encoder_create: ") + hipGetErrorString(e));
  }
  *out = h;
  return SW_OK;
}

// Every stream this encoder has work on, idle: its own (launch, copy-in, copy-out, merge forks) and
// the caller's stream of its last device-entry launch (its ws_done event, recorded after that
// launch's last kernel and after the finder's).  Before anything is freed or unpinned: round 4's
// destroy freed first and synchronised only the launch stream.  Other encoders and
// the caller's unrelated work are not waited for.
static hipError_t drain_own(sw_encoder* h) {
  hipError_t e = hipSuccess;
  auto take = [&](hipError_t x) { if (e == hipSuccess) e = x; };
  if (h->ws_done) take(hipEventSynchronize(h->ws_done));
  for (hipStream_t s : {h->stream, h->s_h2d, h->s_d2h, h->s_fork[0], h->s_fork[1]})
    if (s) take(hipStreamSynchronize(s));
  return e;
}

extern "C" void sw_encoder_destroy(sw_encoder* h) {
  if (!h) return;
  {
    DeviceGuard g(h->device);
    (void)drain_own(h);  // (every stream of this encoder idle before anything is freed or unpinned)
    free_workspace(h);
    free_io(h);
    if (h->ws_done) (void)hipEventSynchronize(h->ws_done);
    free_pipe(h);
    for (const auto& r : h->pins) (void)hipHostUnregister((void*)((uintptr_t)r.h & ~(uintptr_t)4095));
    h->pins.clear();
    (void)hipFree(h->d_done);
    delete h->pool;
    if (h->s_h2d) (void)hipStreamDestroy(h->s_h2d);
    if (h->s_d2h) (void)hipStreamDestroy(h->s_d2h);
    for (int k = 0; k < 2; ++k) {
      if (h->s_fork[k]) (void)hipStreamDestroy(h->s_fork[k]);
      if (h->ev_join[k]) (void)hipEventDestroy(h->ev_join[k]);
    }
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_fork_long) (void)hipEventDestroy(h->ev_fork_long);
    (void)hipFree(h->d_spt);
    (void)hipFree(h->d_spf);
    (void)hipFree(h->d_spf_list);
    (void)hipFree(h->d_spf_off);
    (void)hipFree(h->d_nsp);
    (void)hipFree(h->d_table);
    (void)hipFree(h->d_chunks);
    (void)hipFree(h->d_inv);
    if (h->ws_done) (void)hipEventDestroy(h->ws_done);
    if (h->h_ddfull) (void)hipHostFree(h->h_ddfull);
    for (hipEvent_t ev : h->ev_pool) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : h->ev_cls) (void)hipEventDestroy(ev);
    if (h->stream) (void)hipStreamDestroy(h->stream);
  }
  delete h;
}

extern "C" int32_t sw_encoder_pin_host(sw_encoder* h, void* ptr, int64_t bytes) {
  if (!h || !ptr || bytes <= 0) return fail(SW_ERR_ARG, "sw_encoder_pin_host: bad arguments");
  DeviceGuard g(h->device);
  for (const auto& r : h->pins)  // (whole pages: two ranges may not share one)
    if (((uintptr_t)ptr >> 12) <= (((uintptr_t)r.h + r.n - 1) >> 12) && (((uintptr_t)ptr + bytes - 1) >> 12) >= ((uintptr_t)r.h >> 12))
      return fail(SW_ERR_ARG, "sw_encoder_pin_host: shares a page with a pinned range");
  // (whole pages registered: a large numpy / malloc block starts 16 bytes into its first page)
  const uintptr_t pg = 4096, a0 = (uintptr_t)ptr & ~(pg - 1), a1 = ((uintptr_t)ptr + (uintptr_t)bytes + pg - 1) & ~(pg - 1);
  HIP_TRY(hipHostRegister((void*)a0, (size_t)(a1 - a0), hipHostRegisterMapped));
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, (void*)a0, 0);
  if (e != hipSuccess) {
    (void)hipHostUnregister((void*)a0);
    return fail(SW_ERR_HIP, std::string("sw_encoder_pin_host: ") + hipGetErrorString(e));
  }
  h->pins.push_back(sw_encoder::Pinned{(char*)ptr, bytes, (char*)d + ((uintptr_t)ptr - a0)});
  return SW_OK;
}

extern "C" int32_t sw_encoder_unpin_host(sw_encoder* h, void* ptr) {
  if (!h || !ptr) return fail(SW_ERR_ARG, "sw_encoder_unpin_host: bad arguments");
  DeviceGuard g(h->device);
  for (size_t i = 0; i < h->pins.size(); ++i) {
    if (h->pins[i].h != (char*)ptr) continue;
    // (nothing of this encoder may still read or write it -- a write into the range still in flight
    // when its mapping goes faults the device -- and only this encoder's streams touch its pins)
    HIP_TRY(drain_own(h));
    HIP_TRY(hipHostUnregister((void*)((uintptr_t)ptr & ~(uintptr_t)4095)));
    h->pins.erase(h->pins.begin() + (long)i);
    return SW_OK;
  }
  return fail(SW_ERR_ARG, "sw_encoder_unpin_host: not a pinned range");
}

extern "C" int32_t sw_encoder_reserve(sw_encoder* h, int64_t max_bytes, int64_t max_strings) {
  if (!h || max_bytes < 0 || max_strings < 0) return fail(SW_ERR_ARG, "sw_encoder_reserve: bad arguments");
  DeviceGuard g(h->device);
  return ensure_workspace(h, max_bytes);
}

extern "C" int32_t sw_encoder_set_option(sw_encoder* h, int32_t option, int64_t value) {
  if (!h) return fail(SW_ERR_ARG, "sw_encoder_set_option: null handle");
  switch (option) {
    case SW_OPT_CHUNK_TABLE: h->chunks.enabled = value ? 1u : 0u; return SW_OK;
    case SW_OPT_DEDUPE: h->dedupe = value != 0; return SW_OK;
    case SW_OPT_PATTERN:
      if (value != SW_PAT_CL100K && value != SW_PAT_GPT2 && value != SW_PAT_NONE) return fail(SW_ERR_ARG, "bad pattern");
      h->pattern = (int32_t)value;
      return SW_OK;
    case SW_OPT_HOST_PRESPLIT: h->host_presplit = value != 0; return SW_OK;
    case SW_OPT_DEDUPE_SLOTS:
      if (value != 0 && (value < 8 || (value & (value - 1)))) return fail(SW_ERR_ARG, "dedupe slots: 0 or a power of two >= 8");
      h->dedupe_slots = value;
      return SW_OK;
    case SW_OPT_DEDUPE_FP_BITS:
      if (value < 0 || value > 26) return fail(SW_ERR_ARG, "dedupe fingerprint bits: 0..26");
      h->dedupe_fp_mask = (uint32_t)((1ULL << value) - 1);
      return SW_OK;
    case SW_OPT_DEDUPE_EXACT: h->dedupe_exact = value != 0; return SW_OK;
    case SW_OPT_LONG_SPLIT: h->long_split = value != 0; return SW_OK;
    case SW_OPT_PIPE_COPY_KERNELS: h->pipe_kcopy = value != 0; return SW_OK;
    case SW_OPT_MERGE_STREAMS: h->merge_fork = value != 0; return SW_OK;
    case SW_OPT_FUSED_PRESPLIT: h->fused_presplit = value != 0; return SW_OK;
    case SW_OPT_TEST_FAIL_GROWTH: h->test_fail_grow = value ? 1 : 0; h->dd_grow_stop = false; return SW_OK;
    case SW_OPT_DEVICE_SPECIALS: h->device_specials = value != 0; return SW_OK;
    case SW_OPT_STAGED_HEADS:
      if (value < 0 || value > 2) return fail(SW_ERR_ARG, "staged heads: 0 (automatic), 1 (always) or 2 (never)");
      h->staged_heads = (int)value;
      return SW_OK;
    case SW_OPT_COMPACT_KERNEL:
      if (value < 0 || value > 3) return fail(SW_ERR_ARG, "SW_OPT_COMPACT_KERNEL: 0 .. 3");
      h->compact_kernel = (int)value;
      return SW_OK;
    case SW_OPT_PIPE_DEPTH:
      if (value < 2 || value > 4) return fail(SW_ERR_ARG, "pipeline depth: 2 .. 4");
      h->pipe_depth = (int)value;
      return SW_OK;
    case SW_OPT_PIPE_RUN_BYTES:
      if (value != 0 && value < 64) return fail(SW_ERR_ARG, "pipeline run bytes: 0 (off) or >= 64");
      h->pipe_run = std::min<int64_t>(value, kMaxLaunchBytes);
      return SW_OK;
    case SW_OPT_MAX_LAUNCH_BYTES:
      if (value != 0 && (value < 64 || value > kMaxLaunchBytes))
        return fail(SW_ERR_ARG, "max launch bytes: 0 (default) or 64 .. 2^30 - 64");
      h->max_launch = value ? value : kMaxLaunchBytes;
      return SW_OK;
    default: return fail(SW_ERR_ARG, "sw_encoder_set_option: unknown option");
  }
}

extern "C" int64_t sw_encoder_get_info(const sw_encoder* h, int32_t what) {
  if (!h) return SW_ERR_ARG;
  switch (what) {
    case SW_INFO_MERGES: return h->n_merges;
    case SW_INFO_CHUNK_ENTRIES: return h->n_chunk_entries;
    case SW_INFO_WIDE_TABLE: return h->table.wide;
    case SW_INFO_IDS16: return h->ids16 ? 1 : 0;
    case SW_INFO_SPLIT: return h->split_ok ? 1 : 0;
    case SW_INFO_DEDUPE_SLOTS: return h->dd_slots;
    case SW_INFO_CHUNK_TABLE_BYTES: return h->chunk_table_bytes;
    default: return SW_ERR_ARG;
  }
}

extern "C" int32_t sw_encoder_set_timing(sw_encoder* h, int32_t on) {
  if (!h) return fail(SW_ERR_ARG, "sw_encoder_set_timing: null handle");
  h->timing = on != 0;
  h->ev_used = 0;
  h->ev_cls_used = 0;
  return SW_OK;
}

// Average device time of the classification kernel alone (k_split_classify, or k_classify with a
// caller's bitmap) over the launches recorded since the last sw_encoder_set_timing(h, 1): the
// pipeline's dominant kernel, for the per-kernel roofline (HIP events on the launch stream).
extern "C" double sw_encoder_last_classify_ms(const sw_encoder* h) {
  if (!h || h->ev_cls_used == 0) return -1.0;
  DeviceGuard g(h->device);
  if (hipEventSynchronize(h->ev_cls[2 * h->ev_cls_used - 1]) != hipSuccess) return -1.0;
  double sum = 0;
  for (size_t i = 0; i < h->ev_cls_used; ++i) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, h->ev_cls[2 * i], h->ev_cls[2 * i + 1]) != hipSuccess) return -1.0;
    sum += ms;
  }
  return sum / (double)h->ev_cls_used;
}

// Average device time of the whole sw_encode_device pipeline (k_tile_strings .. k_string_offsets) over the
// launches recorded since the last sw_encoder_set_timing(h, 1); synchronises on the last recorded event.
extern "C" double sw_encoder_last_kernel_ms(const sw_encoder* h) {
  if (!h || h->ev_used == 0) return -1.0;
  DeviceGuard g(h->device);
  if (hipEventSynchronize(h->ev_pool[2 * h->ev_used - 1]) != hipSuccess) return -1.0;
  double sum = 0;
  for (size_t i = 0; i < h->ev_used; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->ev_pool[2 * i], h->ev_pool[2 * i + 1]) != hipSuccess) return -1.0;
    sum += ms;
  }
  return sum / (double)h->ev_used;
}

// Diagnostic builds only (-DSW_STAMPS): cycles per pipeline phase summed over workgroups
// since the workspace was allocated (or the last reset).
extern "C" int32_t sw_encoder_phase_cycles(sw_encoder* h, double* out32, int32_t reset) {
#ifdef SW_STAMPS
  if (!h || !out32 || !h->d_stamps) return fail(SW_ERR_ARG, "sw_encoder_phase_cycles: no workspace");
  DeviceGuard g(h->device);
  std::vector<unsigned long long> v(32 * 64);
  HIP_TRY(hipStreamSynchronize(h->stream));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(v.data(), h->d_stamps, sizeof(unsigned long long) * v.size(), hipMemcpyDeviceToHost));
  for (int i = 0; i < 32; ++i) {
    double sum = 0;
    for (int c = 0; c < 64; ++c) sum += (double)v[i * 64 + c];
    out32[i] = sum;
  }
  if (reset) HIP_TRY(hipMemset(h->d_stamps, 0, sizeof(unsigned long long) * v.size()));
  return SW_OK;
#else
  (void)h; (void)out32; (void)reset;
  return fail(SW_ERR_ARG, "sw_encoder_phase_cycles: not a diagnostic (SW_STAMPS) build");
#endif
}

namespace {
// the long-chunk split + verify passes (long_split.h) on stream s: well-formed tables only
template <bool kWide, bool k16>
hipError_t launch_long_split(sw_encoder* h, hipStream_t s, const EncArgs& a, int part) {
  LongArgs& L = h->lp;
  const dim3 g(kLpGrid), b(kThreads);
  if (part == 2) {  // (the passes that write res, where k_classify's tile-local queue lives until k_scatter)
    hipLaunchKernelGGL((k_lp_fallback<kWide, k16>), g, dim3(64), 0, s, a, L);
    hipLaunchKernelGGL(k_lp_gather, g, b, 0, s, a, L);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_dscan_reduce, dim3(kDscanGrid), b, 0, s, L.lnp, L.lcap, &L.ctl[kLcLong], h->d_lpart);
  hipLaunchKernelGGL(k_dscan_parts, dim3(1), dim3(kDscanGrid), 0, s, h->d_lpart, &L.ctl[kLcPieces]);
  hipLaunchKernelGGL(k_dscan_apply, dim3(kDscanGrid), b, 0, s, L.lnp, L.lcap, &L.ctl[kLcLong], h->d_lpart, L.lpo);
  hipLaunchKernelGGL(k_lp_fill, g, b, 0, s, L);
  hipLaunchKernelGGL((k_lp_encode<kWide, k16>), g, b, 0, s, a, L);  // (and round 0's junctions)
  for (int r = 0; r < kLpRounds; ++r) {
    hipLaunchKernelGGL(k_lp_heads, g, b, 0, s, L, r);
    hipLaunchKernelGGL((k_lp_windows<kWide, k16>), g, b, 0, s, a, L, r);
    hipLaunchKernelGGL((k_lp_bigwin<kWide, k16>), g, dim3(64), 0, s, a, L, r);
    hipLaunchKernelGGL((k_lp_junctions<kWide>), g, b, 0, s, a, L, r + 1);  // (r + 1 == kLpRounds: the final check)
  }
  return hipGetLastError();
}

// every long chunk (> kShort bytes) on stream s, listed from the queue (k_lp_prep): split +
// verify over the whole GPU (long_split.h; well-formed tables), or the wave loop per chunk.
// (Started from the bitmap right after the pre-split, beside k_classify, they only slowed it
// down by as much: both fill the chip.  They run beside the merge kernels, which leave it
// mostly idle.)
// part 1 right after k_classify (its long list and the complete bitmap); part 2, the passes that
// write res, after k_scatter has consumed the tile-local queue aliased there (a.qtmp)
template <bool kWide, bool k16>
hipError_t launch_long(sw_encoder* h, hipStream_t s, const EncArgs& a, bool split, int part) {
  constexpr unsigned kLongGrid = 32768;  // k_merge_long_lds: a workgroup per long chunk (grid-stride past that)
  LongArgs& L = h->lp;
  if (part == 2) {
    if (split) return launch_long_split<kWide, k16>(h, s, a, 2);
    hipLaunchKernelGGL((k_merge_long_lds<kWide, k16>), dim3(kLongGrid), dim3(64), 0, s, a);
    hipLaunchKernelGGL((k_merge_long<kWide>), dim3(512), dim3(kThreads), 0, s, a);  // (over kLongLds bytes)
    return hipGetLastError();
  }
  hipError_t e = hipMemsetAsync(L.ctl, 0, sizeof(int64_t) * kLcAlloc, s);
  if (e == hipSuccess) e = hipMemsetAsync(h->d_big, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lp_prep, dim3(kLpPrepGrid), dim3(kThreads), 0, s, a, L, split ? (int64_t)kShort : INT64_MAX);
  if (!split) return hipGetLastError();
  e = launch_long_split<kWide, k16>(h, s, a, 1);
#ifdef SW_LP_DEBUG
  if (e == hipSuccess && getenv("SW_LP_DEBUG")) {
    int64_t c[kLcAlloc];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(c, L.ctl, sizeof(c), hipMemcpyDeviceToHost);
    fprintf(stderr, "lp: long %lld pieces %lld fall %lld\n", (long long)c[kLcLong], (long long)c[kLcPieces],
            (long long)c[kLcFall]);
    for (int r = 0; r <= kLpRounds; ++r)
      fprintf(stderr, "lp r%d: jun %lld conf %lld heads %lld big %lld big_bytes %lld big_max %lld\n", r,
              (long long)c[kLcJun + r], (long long)c[kLcConf + r], (long long)c[kLcHead + r], (long long)c[kLcBig + r],
              r < kLpRounds ? (long long)c[kLcDbg + r] : 0LL, r < kLpRounds ? (long long)c[kLcDbg + kLpRounds + r] : 0LL);
  }
#endif
  return e;
}

// special-token occurrences of one launch, on the device (sw_encode_ex)
struct DevSpecials {
  const int64_t* pos = nullptr;
  const int32_t* len = nullptr;
  const int32_t* id = nullptr;
  int64_t n = 0;                    // the count, or (n_dev given) the arrays' capacity
  const int64_t* n_dev = nullptr;   // the count in device memory (sw_find_specials_device)
};

// the device pipeline; d_out_ids is int32_t*, or uint16_t* when out16 (the table is ids16)
// A launch whose dedupe table overflowed (chunks that found all 8 candidates of their line taken,
// counted by the device and published to host memory by k_string_offsets) grows the table for
// the launches after it: to the power of two >= 2 x (entries + overflow), at most kDdSlotsMax.
// The count is read without waiting: a launch still running is seen by a later call.
// The new table is allocated beside the old one and swapped in only when all three buffers exist:
// growth is an optimisation, so an allocation failure keeps the table that works (and stops
// further attempts on this handle) instead of leaving the handle half-built.
// The entries of the dedupe table a launch of n bytes uses: a prefix sized for its bytes -- 2^16 at
// least, one per 8 input bytes, at most what is allocated -- so that a small launch after a large
// one, or after the table has grown for a low-repetition corpus, clears kilobytes instead of the
// whole table (the 1 GiB launches use all of it: 2^22 entries by default, 2^24 grown)
int64_t launch_dd_slots(const sw_encoder* h, int64_t n_bytes) {
  int64_t want = 1LL << 16;
  while (want < n_bytes / 8 && want < h->dd_slots) want <<= 1;
  return std::min<int64_t>(want, h->dd_slots);
}

int32_t grow_dedupe(sw_encoder* h, int64_t n_bytes) {
  if (launch_dd_slots(h, n_bytes) < h->dd_slots) return SW_OK;  // (a prefix launch: more entries would not serve it)
  const unsigned long long over = h->h_ddfull ? __atomic_load_n(h->h_ddfull, __ATOMIC_ACQUIRE) : 0ULL;
  constexpr int64_t kGrowDiv = 32;  // (grow when more than slots / this many chunks found no entry)
  if (!h->d_dtab || h->dedupe_slots || h->dd_grow_stop || over <= (unsigned long long)(h->dd_slots / kGrowDiv) ||
      h->dd_slots >= kDdSlotsMax)
    return SW_OK;  // (SW_OPT_DEDUPE_SLOTS caps the table on purpose: no growth)
  int64_t slots = h->dd_slots;
  while (slots < 2 * (h->dd_slots + (int64_t)over) && slots < kDdSlotsMax) slots <<= 1;
  uint64_t* dtab = nullptr;
  uint4* dres = nullptr;
  uint8_t* dcnt = nullptr;
  bool ok = !h->test_fail_grow;
  ok = ok && hipMalloc(&dtab, sizeof(uint64_t) * kDdWords * (slots)) == hipSuccess;
  ok = ok && hipMalloc(&dres, sizeof(uint4) * (slots)) == hipSuccess;
  ok = ok && hipMalloc(&dcnt, slots) == hipSuccess;
  __atomic_store_n(h->h_ddfull, 0ULL, __ATOMIC_RELEASE);
  if (!ok) {
    if (dtab) (void)hipFree(dtab);
    if (dres) (void)hipFree(dres);
    if (dcnt) (void)hipFree(dcnt);
    (void)hipGetLastError();  // (the failed allocation's status: not this launch's error)
    h->dd_grow_stop = true;
    return SW_OK;
  }
  // the old table may still be in use by the previous launch
  if (h->ws_pending) HIP_TRY(hipEventSynchronize(h->ws_done));
  (void)hipFree(h->d_dtab); (void)hipFree(h->d_dres); (void)hipFree(h->d_dcnt);
  h->d_dtab = dtab; h->d_dres = dres; h->d_dcnt = dcnt;
  h->dd_slots = slots;
  h->dmask = (uint32_t)(slots - 1);
  return SW_OK;
}

// the specials' table on the device (rebuilt only when the specials change)
int32_t set_specials(sw_encoder* h, const sw_specials* sp) {
  if (sp && sp->n > 0 && (!sp->bytes || !sp->off || !sp->ids)) return fail(SW_ERR_ARG, "specials: null arrays");
  const int64_t n = sp ? sp->n : 0;
  std::string key;
  if (n > 0) {
    if (sp->off[0] < 0) return fail(SW_ERR_ARG, "specials: bad offsets");
    for (int64_t k = 0; k < n; ++k)
      if (sp->off[k + 1] < sp->off[k]) return fail(SW_ERR_ARG, "specials: bad offsets");
    const int64_t nb = sp->off[n];
    if (nb > INT32_MAX / 2 || n > INT32_MAX / 8) return fail(SW_ERR_ARG, "specials: too large");
    key.assign((const char*)&n, sizeof(n));
    key.append((const char*)sp->off, sizeof(int64_t) * (size_t)(n + 1));
    key.append((const char*)sp->ids, sizeof(int32_t) * (size_t)n);
    key.append((const char*)sp->bytes, (size_t)nb);
  }
  if (h->d_spt && key == h->spt_key) return SW_OK;
  DeviceGuard g(h->device);
  if (h->ws_pending) HIP_TRY(hipEventSynchronize(h->ws_done));  // (a finder still reading the old table)
  (void)hipFree(h->d_spt);
  h->d_spt = nullptr;
  h->spt = SpTab{};
  h->spt_key.clear();
  h->spt_dev = false;
  if (n == 0) return SW_OK;
  const int64_t b0 = sp->off[0], nb = sp->off[n] - b0;
  std::vector<int32_t> off((size_t)n + 1), ids((size_t)n), list, first(257, 0);
  for (int64_t k = 0; k <= n; ++k) off[(size_t)k] = (int32_t)(sp->off[k] - b0);
  for (int64_t k = 0; k < n; ++k) ids[(size_t)k] = sp->ids[k];
  std::vector<std::vector<int32_t>> by_first(256);
  int32_t max_len = 0, min_len = INT32_MAX;
  const bool few = n <= 255;  // (the one-pass finder records a special's index in a byte)
  for (int64_t k = 0; k < n; ++k) {
    const int32_t L = off[(size_t)k + 1] - off[(size_t)k];
    if (L == 0) continue;  // (an empty special never matches)
    by_first[sp->bytes[sp->off[k]]].push_back((int32_t)k);
    max_len = std::max(max_len, L);
    min_len = std::min(min_len, L);
  }
  SpTab t{};
  uint32_t fb = 0;
  for (int b = 0; b < 256; ++b) {
    first[(size_t)b] = (int32_t)list.size();
    if (by_first[(size_t)b].empty()) continue;
    t.filt[b >> 5] |= 1u << (b & 31);
    if (t.n_first < kSpMaxFirstSwar) fb |= (uint32_t)b << (8 * t.n_first);
    ++t.n_first;
    list.insert(list.end(), by_first[(size_t)b].begin(), by_first[(size_t)b].end());
  }
  first[256] = (int32_t)list.size();
  if (list.empty()) list.push_back(0);
  t.fb = fb;
  t.max_len = max_len;
  t.n = (int32_t)n;
  // the LDS image of k_sp_find (specials_find.h, above sft_len), when the finder takes the table
  std::vector<uint32_t> img;
  if (few && max_len <= kSpMaxLen) {
    const int32_t n_list = first[256];
    t.o_first = (int32_t)n;
    t.o_rec = (t.o_first + 129 + 3) & ~3;  // (16-byte aligned records)
    t.o_tag = t.o_rec + kSfRecWords * n_list;
    t.o_words = t.o_tag + n_list;
    img.assign((size_t)t.o_words, 0u);
    for (int b = 0; b <= 256; ++b) img[(size_t)t.o_first + b / 2] |= (uint32_t)first[(size_t)b] << (16 * (b & 1));
    std::vector<uint32_t> wo_of((size_t)n, 0u);
    for (int64_t k = 0; k < n; ++k) {
      const int32_t L = off[(size_t)k + 1] - off[(size_t)k];
      const size_t wo = img.size() - (size_t)t.o_words;
      wo_of[(size_t)k] = (uint32_t)wo;
      img[(size_t)k] = (uint32_t)wo | (uint32_t)L << 16;
      img.resize(img.size() + (size_t)(L + 3) / 4, 0u);
      std::memcpy(img.data() + t.o_words + wo, sp->bytes + sp->off[k], (size_t)L);
    }
    for (int32_t g = 0; g < n_list; ++g) {
      const int32_t k = list[(size_t)g], L = off[(size_t)k + 1] - off[(size_t)k];
      uint32_t* rec = img.data() + t.o_rec + kSfRecWords * g;
      for (int32_t j = 0; j < std::min<int32_t>(L, 16); ++j) {
        rec[j / 4] |= (uint32_t)sp->bytes[sp->off[k] + j] << (8 * (j % 4));
        rec[4 + j / 4] |= 0xFFu << (8 * (j % 4));
      }
      img[(size_t)t.o_tag + g] = (uint32_t)k | (uint32_t)L << 8 | wo_of[(size_t)k] << 16;
    }
    img.push_back(0u);  // (k_sp_find reads a special's second word even for one of <= 4 bytes)
    t.img_words = (int32_t)img.size();
  }
  // one buffer: bytes | off | ids | list | first | LDS image
  const size_t o_off = ((size_t)nb + 15) & ~(size_t)15, o_ids = o_off + 4 * off.size(), o_list = o_ids + 4 * ids.size(),
               o_first = o_list + 4 * list.size(), o_img = o_first + 4 * first.size(), total = o_img + 4 * img.size();
  std::vector<char> host(total, 0);
  std::memcpy(host.data(), sp->bytes + b0, (size_t)nb);
  std::memcpy(host.data() + o_off, off.data(), 4 * off.size());
  std::memcpy(host.data() + o_ids, ids.data(), 4 * ids.size());
  std::memcpy(host.data() + o_list, list.data(), 4 * list.size());
  std::memcpy(host.data() + o_first, first.data(), 4 * first.size());
  if (!img.empty()) std::memcpy(host.data() + o_img, img.data(), 4 * img.size());
  HIP_TRY(hipMalloc(&h->d_spt, total));
  HIP_TRY(hipMemcpy(h->d_spt, host.data(), total, hipMemcpyHostToDevice));
  char* d = (char*)h->d_spt;
  t.bytes = (const uint8_t*)d;
  t.off = (const int32_t*)(d + o_off);
  t.ids = (const int32_t*)(d + o_ids);
  t.list = (const int32_t*)(d + o_list);
  t.first = (const int32_t*)(d + o_first);
  t.img = img.empty() ? nullptr : (const uint32_t*)(d + o_img);
  h->spt = t;
  h->spt_key = key;
  h->spt_dev = t.n_first > 0 && max_len <= kSpMaxLen && few;
  h->spt_min_len = t.n_first > 0 ? min_len : 1;
  return SW_OK;
}

// the occurrences of the handle's specials in d_bytes (sw_find_specials_device), on stream st
int32_t find_specials_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                             int64_t n_str, int64_t* d_pos, int32_t* d_len, int32_t* d_id, int64_t cap, int64_t* d_count,
                             hipStream_t st) {
  if (!h || n_bytes < 0 || n_str < 0 || !d_str_off || !d_count || (n_bytes > 0 && !d_bytes))
    return fail(SW_ERR_ARG, "sw_find_specials_device: bad arguments");
  if (n_bytes > kMaxLaunchBytes) return fail(SW_ERR_ARG, "sw_find_specials_device: n_bytes > 2^30 - 64");
  if (h->d_spt && h->spt.n_first > 0 && !h->spt_dev)
    return fail(SW_ERR_ARG, "sw_find_specials_device: a special over 64 bytes, or over 255 specials (use the host finder)");
  if (h->spt.n_first > 0 && n_bytes > 0 && (cap < n_bytes / h->spt_min_len || !d_pos || !d_len || !d_id))
    return fail(SW_ERR_CAP, "sw_find_specials_device: cap < n_bytes / (shortest special's length)");
  if (h->ws_pending && h->ws_stream != st) HIP_TRY(hipStreamWaitEvent(st, h->ws_done, 0));
  const int64_t n_tiles = (n_bytes + kTile - 1) / kTile;
  if (h->spt.n_first == 0 || n_tiles == 0) {
    HIP_TRY(hipMemsetAsync(d_count, 0, sizeof(int64_t), st));
  } else {
    int32_t rc = ensure_workspace(h, n_bytes);
    if (rc) return rc;
    const int64_t tcap = kTile / h->spt_min_len + 1;  // (a tile's occurrences: at most this many)
    const int64_t n_parts = (n_tiles + kScanBlock - 1) / kScanBlock + 1;
    if (n_tiles > h->spf_tiles || tcap > h->spf_tcap) {
      (void)hipFree(h->d_spf); (void)hipFree(h->d_spf_list); (void)hipFree(h->d_spf_off);
      h->d_spf = nullptr; h->d_spf_list = nullptr; h->d_spf_off = nullptr; h->spf_tiles = 0; h->spf_tcap = 0;
      HIP_TRY(hipMalloc(&h->d_spf, sizeof(uint32_t) * ((size_t)n_tiles * (2 * 64 + 2) + 1)));
      HIP_TRY(hipMalloc(&h->d_spf_list, sizeof(uint32_t) * (size_t)n_tiles * (size_t)tcap));
      HIP_TRY(hipMalloc(&h->d_spf_off, sizeof(int64_t) * (size_t)(2 * (n_tiles + n_parts) + 1)));
      h->spf_tiles = n_tiles;
      h->spf_tcap = tcap;
    }
    SpFind f;
    f.bytes = d_bytes; f.n_bytes = n_bytes; f.str_off = d_str_off; f.n_str = n_str;
    f.tile_slo = h->d_tile_slo; f.n_tiles = n_tiles;
    f.cbits = h->d_spf; f.chosen = h->d_spf + 64 * n_tiles;
    f.tcand = h->d_spf + 128 * n_tiles; f.tcnt = f.tcand + n_tiles;
    f.flag = (unsigned int*)(f.tcnt + n_tiles);
    f.list = h->d_spf_list; f.tcap = tcap;
    int64_t* toff = h->d_spf_off;                     // [n_tiles] + partials
    int64_t* toff2 = h->d_spf_off + n_tiles + n_parts;  // the global path's
    int64_t* total2 = toff2 + n_tiles + n_parts;
    const dim3 gw((unsigned)((n_tiles + kWaves - 1) / kWaves)), bw(kThreads);
    HIP_TRY(hipMemsetAsync(f.flag, 0, sizeof(unsigned int), st));
    hipLaunchKernelGGL(k_tile_strings, dim3((unsigned)((n_tiles + 255) / 256)), dim3(256), 0, st, d_str_off, n_str,
                       n_tiles, h->d_tile_slo, nullptr);
    const bool swar = h->spt.n_first <= kSpMaxFirstSwar;
    // the one-pass path
    const size_t lds_tab = sizeof(uint32_t) * (size_t)h->spt.img_words;
    if (swar) hipLaunchKernelGGL(k_sp_find<true>, gw, bw, lds_tab, st, h->spt, f);
    else hipLaunchKernelGGL(k_sp_find<false>, gw, bw, lds_tab, st, h->spt, f);
    HIP_TRY(launch_scan(st, f.tcnt, n_tiles, toff + n_tiles, toff, d_count));
    const dim3 ge((unsigned)((n_tiles + kWaves * kSfEmitTiles - 1) / (kWaves * kSfEmitTiles)));
    hipLaunchKernelGGL(k_sp_emit, ge, bw, 0, st, h->spt, f, (const int64_t*)toff, d_pos, d_len, d_id);
    // the global-memory path: its kernels return at once unless k_sp_find raised the flag (small
    // grids that loop over the tiles)
    const dim3 gg(std::min<unsigned>(gw.x, kSfGlobalBlocks));
    if (swar) hipLaunchKernelGGL(k_sp_detect<true>, gg, bw, 0, st, h->spt, f);
    else hipLaunchKernelGGL(k_sp_detect<false>, gg, bw, 0, st, h->spt, f);
    hipLaunchKernelGGL(k_sp_resolve, gg, bw, lds_tab, st, h->spt, f);
    hipLaunchKernelGGL(k_sp_count, gg, bw, 0, st, f);
    HIP_TRY(launch_scan(st, f.tcnt, n_tiles, toff2 + n_tiles, toff2, total2));
    hipLaunchKernelGGL(k_sp_write, gg, bw, 0, st, h->spt, f, (const int64_t*)toff2, d_pos, d_len, d_id);
    hipLaunchKernelGGL(k_sp_fix_count, dim3(1), dim3(64), 0, st, (const unsigned int*)f.flag, (const int64_t*)total2,
                       d_count);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(h->ws_done, st));
  h->ws_stream = st;
  h->ws_pending = true;
  return SW_OK;
}

int32_t encode_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off, int64_t n_str,
                      const uint64_t* d_chunk_bits, const DevSpecials& sp, void* d_out_ids, bool out16,
                      int64_t* d_out_off, void* stream, int64_t* n_tokens_host, int32_t pattern_call = -1) {
  if (pattern_call < -1 || pattern_call > SW_PAT_NONE) return fail(SW_ERR_ARG, "sw_encode_device: unknown pattern");
  if (!h || n_bytes < 0 || n_str < 0 || !d_str_off || !d_out_off || (n_bytes > 0 && (!d_bytes || !d_out_ids)))
    return fail(SW_ERR_ARG, "sw_encode_device: bad arguments");
  if (sp.n < 0 || (sp.n > 0 && (!sp.pos || !sp.len || !sp.id)))
    return fail(SW_ERR_ARG, "sw_encode_device: bad special-token occurrences");
  if (out16 && !h->ids16) return fail(SW_ERR_ARG, "sw_encode_device: 16-bit output needs a table whose ids fit 16 bits");
  if (out16 && sp.n > 0) return fail(SW_ERR_ARG, "sw_encode_device: 16-bit output with special tokens is not supported");
  if (n_bytes > kMaxLaunchBytes) return fail(SW_ERR_ARG, "sw_encode_device: n_bytes > 2^30 - 64 (split the batch)");
  DeviceGuard g(h->device);
  const int32_t pattern = pattern_call >= 0 ? pattern_call : h->pattern;  // (per call, or the handle's option)
  hipStream_t st = (hipStream_t)stream;  // (NULL: the null stream, as torch's default stream)
  // the workspace belongs to the handle: order this launch after the previous one on any stream
  if (h->ws_pending && h->ws_stream != st) HIP_TRY(hipStreamWaitEvent(st, h->ws_done, 0));
  int32_t rc = ensure_workspace(h, n_bytes);
  if (rc == SW_OK && h->dedupe) rc = grow_dedupe(h, n_bytes);
  if (rc) return rc;
  const int64_t n_tiles = (n_bytes + kTile - 1) / kTile;
  h->last_tiles = n_tiles;
  hipEvent_t e1 = nullptr;
  if (h->timing) {  // the whole device pipeline, k_tile_strings .. k_string_offsets
    while (h->ev_pool.size() < 2 * (h->ev_used + 1)) {
      hipEvent_t ev;
      HIP_TRY(hipEventCreate(&ev));
      h->ev_pool.push_back(ev);
    }
    e1 = h->ev_pool[2 * h->ev_used + 1];
    HIP_TRY(hipEventRecord(h->ev_pool[2 * h->ev_used], st));
  }
  if (n_tiles > 0)  // (the pre-split and k_classify start from each tile's first string)
    hipLaunchKernelGGL(k_tile_strings, dim3((unsigned)((n_tiles + 255) / 256)), dim3(256), 0, st, d_str_off, n_str,
                       n_tiles, h->d_tile_slo, h->d_lcount);  // (and the long list emptied)
  const SpArgs spa{sp.pos, sp.len, sp.id, sp.n, h->d_tile_sp, h->d_tile_sp + (n_tiles + 1)};
  if (n_tiles > 0 && sp.n > 0)  // (... and their first special-token occurrence; the count last)
    hipLaunchKernelGGL(k_tile_specials, dim3((unsigned)((n_tiles + 1 + 255) / 256)), dim3(256), 0, st, sp.pos, sp.len,
                       sp.n, sp.n_dev, n_tiles, h->d_tile_sp, h->d_tile_sp + (n_tiles + 1));
  // the full path (no caller bitmap): the device pre-split, fused into the classification
  // (k_edges + k_split_classify) or as its own kernel first (SW_OPT_FUSED_PRESPLIT 0; special
  // tokens always take the fused kernel)
  const bool fused = n_tiles > 0 && !d_chunk_bits && (h->fused_presplit || sp.n > 0);
  if (n_tiles > 0 && !d_chunk_bits) {
    if (!fused) HIP_TRY(launch_presplit(st, d_bytes, n_bytes, d_str_off, n_str, pattern, h->d_pbits, h->d_tile_slo));
    d_chunk_bits = h->d_pbits;
  }
  if (n_tiles > 0) {
    EncArgs a;
    a.bytes = d_bytes; a.n_bytes = n_bytes; a.bits = d_chunk_bits; a.n_words = (n_bytes + 63) / 64;
    a.str_off = d_str_off; a.n_str = n_str; a.table = h->table; a.chunks = h->chunks;
    a.scratch = h->d_scratch; a.res = h->d_res;
    a.tile_slots = h->d_tile_slots; a.tile_nref = h->d_tile_nref; a.rlist = h->d_rlist; a.tile_cnt = h->d_tile_cnt;
    a.dtab = h->d_dtab; a.dedupe = h->dedupe ? 1u : 0u; a.dfp_mask = h->dedupe_fp_mask;
    {
      const uint32_t lmask = (uint32_t)(launch_dd_slots(h, n_bytes) - 1);
      a.dmask = h->dedupe_slots ? std::min<uint32_t>(lmask, (uint32_t)(h->dedupe_slots - 1)) : lmask;
    }
    a.dexact = h->dedupe_exact ? (uint32_t)kDdExactMax : 0u;
    a.dres = h->d_dres;
    a.dcnt = h->d_dcnt;
    a.dd_full = h->d_ddfull;
    a.llist = h->d_llist; a.l_count = h->d_lcount;
    a.big_count = h->d_big; a.big_list = h->d_big + 1;
    a.out_off = d_out_off; a.tile_slo = h->d_tile_slo;
    a.n_tiles = n_tiles; a.qtmp = h->d_res; a.bcnt = h->d_bcnt; a.boff = h->d_boff; a.q_total = h->d_qtotal;
    a.queue = h->d_queue; a.stamps = h->d_stamps;
    a.inv = h->d_inv; a.n_inv = h->n_inv; a.ids16 = h->ids16 ? 1u : 0u;
    a.lstart = h->lp.wstart; a.llen = h->lp.wlen; a.n_long = &h->lp.ctl[kLcWave]; a.lcap = h->lp.lcap;
    a.sp = spa;
    // the result heads staged by k_tile_count when the dedupe table has grown past the caches (its
    // heads, 16 B an entry, are random HBM reads that k_compact would otherwise make a second time)
    // (automatic: the previous launch ran more than kStagedMinMerges merge loops, i.e. its distinct
    // results' heads spread over more 64-byte lines than the 256 MB Infinity Cache holds -- ENTROPY's
    // 15.6 M per GiB; a GPT-2 pre-split with specials runs 3 M and keeps them cached, and C2 0.75 M.
    // Read without waiting, like the compaction kernel's choice: results are identical either way)
    const unsigned long long prev_merges = h->h_ddfull ? __atomic_load_n(&h->h_ddfull[2], __ATOMIC_RELAXED) : 0ULL;
    a.staged_heads = (h->staged_heads == 1 || (h->staged_heads == 0 && h->dedupe && prev_merges > kStagedMinMerges)) ? 1u : 0u;
    const bool split = h->split_ok && h->long_split;  // (split + verify needs a well-formed table)
    // (cleared per launch rather than entry by entry by the merge kernels that empty the claims:
    // the memset leaves the table's lines in the caches, and the probes then hit -- clearing only
    // the claims made k_split_classify 2% slower on C2, r4n/r4o A/B)
    const size_t dtab_bytes = sizeof(uint64_t) * kDdWords * ((size_t)a.dmask + 1);
    // (k_edges' threads clear the table -- +4 us of k_edges for a 9 us memset on C2, r8b -- when its
    // grid covers the table in a few stores per thread; a small launch after the table has grown
    // for a large one keeps the memset, which is not limited to k_edges' few blocks)
    const int64_t edge_threads = (n_tiles + 1 + 255) / 256 * 256;
    const bool clr_in_edges = fused && dtab_bytes % 16 == 0 && (int64_t)(dtab_bytes / 16) <= 16 * edge_threads;
    if (h->dedupe && !clr_in_edges) HIP_TRY(hipMemsetAsync(h->d_dtab, 0, dtab_bytes, st));
    hipEvent_t c1 = nullptr;  // (timing: the classification kernel alone -- k_split_classify or k_classify)
    if (h->timing) {
      while (h->ev_cls.size() < 2 * (h->ev_cls_used + 1)) {
        hipEvent_t ev;
        HIP_TRY(hipEventCreate(&ev));
        h->ev_cls.push_back(ev);
      }
      c1 = h->ev_cls[2 * h->ev_cls_used + 1];
    }
    auto cls_begin = [&]() -> hipError_t { return c1 ? hipEventRecord(h->ev_cls[2 * h->ev_cls_used], st) : hipSuccess; };
    auto cls_end = [&]() -> hipError_t {
      if (!c1) return hipSuccess;
      ++h->ev_cls_used;
      return hipEventRecord(c1, st);
    };
    if (fused) {
      const PbArgs pg{d_bytes, n_bytes, d_str_off, n_str, h->d_tile_slo, spa};
      hipLaunchKernelGGL(k_edges, dim3((unsigned)((n_tiles + 1 + 255) / 256)), dim3(256), 0, st, pg, n_tiles,
                         (int)pattern, h->d_edge, h->d_redo, h->dedupe && clr_in_edges ? (uint4*)h->d_dtab : nullptr,
                         (int64_t)(dtab_bytes / 16));
      const dim3 gc((unsigned)((n_tiles + kWaves - 1) / kWaves));
      const RedoList redo{h->d_redo, (int64_t*)(h->d_redo + 2)};  // (its count zeroed by k_edges)
      HIP_TRY(cls_begin());
      if (sp.n > 0) {
        hipLaunchKernelGGL(k_split_classify<true>, gc, dim3(kThreads), 0, st, a, pg, (int)pattern,
                           (const uint32_t*)h->d_edge, (uint32_t*)h->d_pbits, redo);
        HIP_TRY(cls_end());
        hipLaunchKernelGGL(k_split_redo<true>, dim3(kRedoGrid), dim3(kThreads), 0, st, a, pg, (int)pattern,
                           (const uint32_t*)h->d_edge, (uint32_t*)h->d_pbits, redo);
      } else {
        hipLaunchKernelGGL(k_split_classify<false>, gc, dim3(kThreads), 0, st, a, pg, (int)pattern,
                           (const uint32_t*)h->d_edge, (uint32_t*)h->d_pbits, redo);
        HIP_TRY(cls_end());
        hipLaunchKernelGGL(k_split_redo<false>, dim3(kRedoGrid), dim3(kThreads), 0, st, a, pg, (int)pattern,
                           (const uint32_t*)h->d_edge, (uint32_t*)h->d_pbits, redo);
      }
    } else {
      // (tiles over k_classify's chunk-start capacity: listed, then classified by k_classify_big)
      unsigned int* ov_count = h->d_redo;
      int64_t* ov_tiles = (int64_t*)(h->d_redo + 2);
      HIP_TRY(hipMemsetAsync(ov_count, 0, sizeof(unsigned int), st));
      const dim3 gc((unsigned)((n_tiles + kWaves - 1) / kWaves));
      HIP_TRY(cls_begin());
      if (sp.n > 0) {
        hipLaunchKernelGGL(k_classify<true>, gc, dim3(kThreads), 0, st, a, ov_count, ov_tiles);
        HIP_TRY(cls_end());
        hipLaunchKernelGGL(k_classify_big<true>, dim3(kRedoGrid), dim3(kThreads), 0, st, a, (const unsigned int*)ov_count,
                           (const int64_t*)ov_tiles);
      } else {
        hipLaunchKernelGGL(k_classify<false>, gc, dim3(kThreads), 0, st, a, ov_count, ov_tiles);
        HIP_TRY(cls_end());
        hipLaunchKernelGGL(k_classify_big<false>, dim3(kRedoGrid), dim3(kThreads), 0, st, a, (const unsigned int*)ov_count,
                           (const int64_t*)ov_tiles);
      }
    }
    HIP_TRY(hipGetLastError());
    // streams of the merge kernels: [0] buckets 17..32 B, then 5..8 B, [1] 9..16 B, then 2..4 B
    // (balanced for the memo-off loads: 9.4 + 6.6 against 12.3 + 3.1 ms), [3] the long chunks,
    // forked right here: they start from k_classify's long list and the complete bitmap, beside
    // the scan and the scatter (C2: their ~20 small passes no longer outlast the merge kernels).
    // (Two forks only: streams beyond the process's hardware queues (4) share one and run in
    // launch order, which put the long chunks behind a bucket.)
    hipStream_t ms[4] = {st, st, st, st};
    if (h->merge_fork) {
      for (int k = 0; k < 2; ++k) {
        if (!h->s_fork[k]) HIP_TRY(hipStreamCreateWithFlags(&h->s_fork[k], hipStreamNonBlocking));
        if (!h->ev_join[k]) HIP_TRY(hipEventCreateWithFlags(&h->ev_join[k], hipEventDisableTiming));
      }
      if (!h->ev_fork) HIP_TRY(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
      if (!h->ev_fork_long) HIP_TRY(hipEventCreateWithFlags(&h->ev_fork_long, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(h->ev_fork_long, st));
      HIP_TRY(hipStreamWaitEvent(h->s_fork[1], h->ev_fork_long, 0));
      ms[1] = h->s_fork[0];
      ms[3] = h->s_fork[1];
    }
    auto long_part = [&](int part) -> hipError_t {
      if (h->table.wide) return launch_long<true, false>(h, ms[3], a, split, part);
      if (h->ids16) return launch_long<false, true>(h, ms[3], a, split, part);
      return launch_long<false, false>(h, ms[3], a, split, part);
    };
    HIP_TRY(long_part(1));
    HIP_TRY(launch_scan(st, h->d_bcnt, kNumBuckets * n_tiles, h->d_part, h->d_boff, h->d_qtotal));
    hipLaunchKernelGGL(k_scatter, dim3((unsigned)((n_tiles + 15) / 16)), dim3(kThreads), 0, st, a);  // (4 tiles a wave)
    const dim3 pg(2048), pb(kThreads);  // persistent grid for the queue kernels
    if (h->merge_fork) {
      HIP_TRY(hipEventRecord(h->ev_fork, st));
      for (int k = 0; k < 2; ++k) HIP_TRY(hipStreamWaitEvent(h->s_fork[k], h->ev_fork, 0));
    }
    HIP_TRY(long_part(2));
    if (h->table.wide) {
      hipLaunchKernelGGL((k_merge_bucket<true, false, 32>), pg, pb, 0, ms[0], a, 8, 9);
      hipLaunchKernelGGL((k_merge_bucket<true, false, 16>), pg, pb, 0, ms[1], a, 5, 7);
      hipLaunchKernelGGL((k_merge_bucket<true, false, 8>), pg, pb, 0, ms[2], a, 3, 4);
      hipLaunchKernelGGL((k_merge_bucket<true, false, 4>), pg, pb, 0, ms[1], a, 0, 2);
    } else if (h->ids16 && h->split_ok) {  // (a well-formed table: the rank-matching loop)
      hipLaunchKernelGGL((k_merge_bucket<false, true, 32, true>), pg, pb, 0, ms[0], a, 8, 9);
      hipLaunchKernelGGL((k_merge_bucket<false, true, 16, true>), pg, pb, 0, ms[1], a, 5, 7);
      hipLaunchKernelGGL((k_merge_bucket<false, true, 8, true>), pg, pb, 0, ms[2], a, 3, 4);
      hipLaunchKernelGGL((k_merge_bucket<false, true, 4, true>), pg, pb, 0, ms[1], a, 0, 2);
    } else if (h->ids16) {
      hipLaunchKernelGGL((k_merge_bucket<false, true, 32>), pg, pb, 0, ms[0], a, 8, 9);
      hipLaunchKernelGGL((k_merge_bucket<false, true, 16>), pg, pb, 0, ms[1], a, 5, 7);
      hipLaunchKernelGGL((k_merge_bucket<false, true, 8>), pg, pb, 0, ms[2], a, 3, 4);
      hipLaunchKernelGGL((k_merge_bucket<false, true, 4>), pg, pb, 0, ms[1], a, 0, 2);
    } else {
      hipLaunchKernelGGL((k_merge_bucket<false, false, 32>), pg, pb, 0, ms[0], a, 8, 9);
      hipLaunchKernelGGL((k_merge_bucket<false, false, 16>), pg, pb, 0, ms[1], a, 5, 7);
      hipLaunchKernelGGL((k_merge_bucket<false, false, 8>), pg, pb, 0, ms[2], a, 3, 4);
      hipLaunchKernelGGL((k_merge_bucket<false, false, 4>), pg, pb, 0, ms[1], a, 0, 2);
    }
    if (h->merge_fork) {
      for (int k = 0; k < 2; ++k) {
        HIP_TRY(hipEventRecord(h->ev_join[k], h->s_fork[k]));
        HIP_TRY(hipStreamWaitEvent(st, h->ev_join[k], 0));
      }
    }
    HIP_TRY(hipGetLastError());
    const dim3 wg((unsigned)((n_tiles + 3) / 4));  // one wave per tile
    if (a.staged_heads)
      hipLaunchKernelGGL(k_tile_count_staged, dim3((unsigned)((n_tiles + kWaves - 1) / kWaves)), dim3(kThreads), 0, st, a);
    else
      hipLaunchKernelGGL(k_tile_count, dim3((unsigned)((n_tiles + kWaves * kTcTiles - 1) / (kWaves * kTcTiles))),
                         dim3(kThreads), 0, st, a);
    HIP_TRY(launch_scan(st, h->d_tile_cnt, n_tiles, h->d_part, h->d_tile_base, h->d_total));
    // the compaction kernel from the last launch's ids per tile (read without waiting: a heuristic)
    int ck = h->compact_kernel;
    if (ck == 0) {
      ck = 1;
      const unsigned long long ids = h->h_ddfull ? __atomic_load_n(&h->h_ddfull[1], __ATOMIC_RELAXED) : 0ULL;
      const unsigned long long tl = (unsigned long long)h->cp_prev_tiles;
      if (tl > 0 && ids > 0) ck = ids <= tl * kCompactTypedMaxIdsPerTile ? 3 : ids <= tl * kCompact7MaxIdsPerTile ? 2 : 1;
    }
    h->cp_prev_tiles = n_tiles;
    if (out16) {
      if (ck == 3) hipLaunchKernelGGL((k_compact7<uint16_t, true>), wg, dim3(kThreads), 0, st, a, h->d_tile_base, (uint16_t*)d_out_ids);
      else if (ck == 2) hipLaunchKernelGGL((k_compact7<uint16_t, false>), wg, dim3(kThreads), 0, st, a, h->d_tile_base, (uint16_t*)d_out_ids);
      else hipLaunchKernelGGL(k_compact<uint16_t>, wg, dim3(kThreads), 0, st, a, h->d_tile_base, (uint16_t*)d_out_ids);
    } else {
      if (ck == 3) hipLaunchKernelGGL((k_compact7<int32_t, true>), wg, dim3(kThreads), 0, st, a, h->d_tile_base, (int32_t*)d_out_ids);
      else if (ck == 2) hipLaunchKernelGGL((k_compact7<int32_t, false>), wg, dim3(kThreads), 0, st, a, h->d_tile_base, (int32_t*)d_out_ids);
      else hipLaunchKernelGGL(k_compact<int32_t>, wg, dim3(kThreads), 0, st, a, h->d_tile_base, (int32_t*)d_out_ids);
    }
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemsetAsync(h->d_total, 0, sizeof(int64_t), st));
  }
  hipLaunchKernelGGL(k_string_offsets, dim3((unsigned)((n_str + 1 + 255) / 256)), dim3(256), 0, st, d_str_off, n_str,
                     n_bytes, h->d_total, d_out_off, h->d_ddfull, h->hd_ddfull, n_tiles > 0 ? h->d_qtotal : nullptr);
  HIP_TRY(hipGetLastError());
  if (h->timing) {
    HIP_TRY(hipEventRecord(e1, st));
    ++h->ev_used;
  }
  HIP_TRY(hipEventRecord(h->ws_done, st));
  h->ws_stream = st;
  h->ws_pending = true;
  if (n_tokens_host) {
    HIP_TRY(hipMemcpyAsync(n_tokens_host, h->d_total, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  return SW_OK;
}

}  // namespace

extern "C" int32_t sw_encode_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                                    int64_t n_str, const uint64_t* d_chunk_bits, int32_t* d_out_ids,
                                    int64_t* d_out_off, void* stream, int64_t* n_tokens_host) {
  return encode_device(h, d_bytes, n_bytes, d_str_off, n_str, d_chunk_bits, DevSpecials{}, d_out_ids, false, d_out_off,
                       stream, n_tokens_host);
}

extern "C" int32_t sw_encode_device_ex(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                                       int64_t n_str, const sw_encode_ex* ex, void* d_out_ids, int64_t* d_out_off,
                                       void* stream, int64_t* n_tokens_host) {
  if (!ex)
    return encode_device(h, d_bytes, n_bytes, d_str_off, n_str, nullptr, DevSpecials{}, d_out_ids, false, d_out_off,
                         stream, n_tokens_host);
  if (ex->struct_size != (int32_t)sizeof(sw_encode_ex))
    return fail(SW_ERR_ARG, "sw_encode_device_ex: struct_size is not sizeof(sw_encode_ex) of this library");
  if (ex->out_bits != 0 && ex->out_bits != 16 && ex->out_bits != 32)
    return fail(SW_ERR_ARG, "sw_encode_device_ex: out_bits 16 or 32");
  if ((ex->flags & SW_EX_PATTERN) && (ex->pattern < SW_PAT_CL100K || ex->pattern > SW_PAT_NONE))
    return fail(SW_ERR_ARG, "sw_encode_device_ex: unknown pattern");
  DevSpecials sp;
  sp.pos = ex->sp_pos; sp.len = ex->sp_len; sp.id = ex->sp_id; sp.n = ex->n_sp; sp.n_dev = ex->d_n_sp;
  if (sp.n_dev && sp.n <= 0) return fail(SW_ERR_ARG, "sw_encode_device_ex: d_n_sp needs n_sp = the arrays' capacity");
  return encode_device(h, d_bytes, n_bytes, d_str_off, n_str, ex->chunk_bits, sp, d_out_ids, ex->out_bits == 16,
                       d_out_off, stream, n_tokens_host, (ex->flags & SW_EX_PATTERN) ? ex->pattern : -1);
}

extern "C" int32_t sw_encoder_set_specials(sw_encoder* h, const sw_specials* sp) {
  if (!h) return fail(SW_ERR_ARG, "sw_encoder_set_specials: null handle");
  return set_specials(h, sp);
}

extern "C" int32_t sw_find_specials_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes,
                                           const int64_t* d_str_off, int64_t n_str, int64_t* d_pos, int32_t* d_len,
                                           int32_t* d_id, int64_t cap, int64_t* d_count, void* stream, int64_t* n_host) {
  if (!h) return fail(SW_ERR_ARG, "sw_find_specials_device: null handle");
  DeviceGuard g(h->device);
  const hipStream_t st = (hipStream_t)stream;
  const int32_t rc = find_specials_device(h, d_bytes, n_bytes, d_str_off, n_str, d_pos, d_len, d_id, cap, d_count, st);
  if (rc) return rc;
  if (n_host) {
    HIP_TRY(hipMemcpyAsync(n_host, d_count, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  return SW_OK;
}

// ids to 16 bits for the device -> host copy (every id of an ids16 table fits)
__global__ void k_pack16(const int32_t* in, const int64_t* total, uint16_t* out) {
  const int64_t n = *total;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint16_t)in[i];
}

// Pipeline copies as kernels over PCIe: a few hundred waves of 16-byte loads keep enough requests
// in flight to run a copy at the link rate (about 57 GB/s each way measured, tools/h2d_probe.hip)
// while the encode kernels run beside them (copy_seg: copy_seg.h, its access ranges checked on the
// CPU by tests/native/copy_seg_emul.cpp).
constexpr int kCopySegs = 6;
struct CopySegs {
  const uint8_t* src[kCopySegs];
  uint8_t* dst[kCopySegs];
  int64_t n[kCopySegs];
};

__global__ void __launch_bounds__(256) k_copy_segs(CopySegs c) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
  for (int k = 0; k < kCopySegs; ++k)
    if (c.n[k] > 0) copy_seg(c.src[k], c.dst[k], c.n[k], t, nt);
}

// one run's results straight into the caller's pinned arrays (sw_encoder_pin_host): its ids as
// int32 at the batch's running count done[0] and its string offsets rebased by it; done[1] set
// (nothing written) if the ids would pass out_cap.  k_push_advance then adds the run's count.
__global__ void __launch_bounds__(256) k_push_direct(const int32_t* __restrict__ ids, const int64_t* ntok,
                                                     const int64_t* d_oo, int64_t n_oo, int32_t* out, int64_t* out_off,
                                                     int64_t out_cap, const int64_t* done) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
  const int64_t n = *ntok, base = done[0];
  if (done[1] || base + n > out_cap) return;
  copy_seg((const uint8_t*)ids, (uint8_t*)(out + base), n * 4, t, nt);
  for (int64_t j = t; j < n_oo; j += nt) out_off[j] = d_oo[j] + base;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope: the host-memory writes leave the caches here)
}
__global__ void k_push_advance(const int64_t* ntok, int64_t out_cap, int64_t* done) {
  if (threadIdx.x != 0) return;
  const int64_t n = *ntok;
  if (done[1] || done[0] + n > out_cap) done[1] = 1;
  else done[0] += n;
}

// one run's results to pinned host memory: ids (16-bit when every id fits, 8 per 16-byte store;
// else 32-bit) and the run's string offsets
__global__ void __launch_bounds__(256) k_push_run(const int32_t* __restrict__ ids, const int64_t* ntok, int wide,
                                                  void* h_ids, const int64_t* d_oo, int64_t n_oo, int64_t* h_oo) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
  const int64_t n = *ntok;
  if (wide) {
    copy_seg((const uint8_t*)ids, (uint8_t*)h_ids, n * 4, t, nt);
  } else {
    const int64_t n8 = n >> 3;
    const v4u32* s = (const v4u32*)ids;
    v4u32* d = (v4u32*)h_ids;
    for (int64_t i = t; i < n8; i += nt) {
      const v4u32 a = __builtin_nontemporal_load(s + 2 * i), b = __builtin_nontemporal_load(s + 2 * i + 1);
      v4u32 o;
      o.x = (a.x & 0xFFFFu) | (a.y << 16);
      o.y = (a.z & 0xFFFFu) | (a.w << 16);
      o.z = (b.x & 0xFFFFu) | (b.y << 16);
      o.w = (b.z & 0xFFFFu) | (b.w << 16);
      d[i] = o;
    }
    uint16_t* d16 = (uint16_t*)h_ids;
    for (int64_t i = (n8 << 3) + t; i < n; i += nt) d16[i] = (uint16_t)ids[i];
  }
  copy_seg((const uint8_t*)d_oo, (uint8_t*)h_oo, n_oo * 8, t, nt);
}

namespace {

// special-token occurrences of a host batch (positions relative to its first byte, ascending)
struct HostSpecials {
  const int64_t* pos = nullptr;
  const int32_t* len = nullptr;
  const int32_t* id = nullptr;
  int64_t n = 0;
  bool narrow = true;  // every id fits the 16-bit download (<= 0xFFFD)
  bool dev = false;    // found on the device, launch by launch (the handle's specials table): pos /
                       // len / id unused, n = 1
};

// the occurrences inside bytes [a, b) of the batch: [*j0, *j1)
void sp_range(const HostSpecials& sp, int64_t a, int64_t b, int64_t* j0, int64_t* j1) {
  *j0 = std::lower_bound(sp.pos, sp.pos + sp.n, a) - sp.pos;
  *j1 = std::lower_bound(sp.pos, sp.pos + sp.n, b) - sp.pos;
}

// 16-bit ids -> the caller's int32 array, 8 at a time with non-temporal stores (the array is written
// once and not read back here: no read-for-ownership of its lines, about a third less host
// memory traffic than plain stores)
static void widen16_stream(const uint16_t* src, int32_t* dst, int64_t n) {
  int64_t i = 0;
  for (; i < n && ((uintptr_t)(dst + i) & 15); ++i) dst[i] = (int32_t)src[i];
  const __m128i z = _mm_setzero_si128();
  for (; i + 8 <= n; i += 8) {
    const __m128i x = _mm_loadu_si128((const __m128i*)(src + i));
    _mm_stream_si128((__m128i*)(dst + i), _mm_unpacklo_epi16(x, z));
    _mm_stream_si128((__m128i*)(dst + i + 4), _mm_unpackhi_epi16(x, z));
  }
  for (; i < n; ++i) dst[i] = (int32_t)src[i];
  _mm_sfence();
}

// sw_encode_batch for a large host batch: runs of whole strings (<= pipe_run bytes, or one longer
// string) through two slots of pinned and device buffers.  Host thread: stage run k (pool copies
// into pinned memory), enqueue its upload and encode, then drain run k - 1 (its 16/32-bit ids and
// offsets to pinned memory, pool copies out to the caller) while run k encodes.
int32_t encode_batch_pipelined(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                               int32_t pattern, const uint64_t* chunk_bits, const HostSpecials& sp, int32_t* out_ids,
                               int64_t out_cap, int64_t* out_off, sw_stats* stats,
                               std::chrono::steady_clock::time_point T0) {
  const bool narrow = h->ids16 && sp.narrow;  // (ids downloaded as 16 bits)
  const int64_t b0 = str_off[0];
  std::vector<std::pair<int64_t, int64_t>> runs;
  int64_t max_b = 1, max_s = 1, max_sp = 1;
  const int64_t run_cap = std::min(h->pipe_run, h->max_launch);  // (a run is one launch)
  for (int64_t s_lo = 0; s_lo < n_str;) {
    int64_t s_hi = s_lo + 1;
    while (s_hi < n_str && str_off[s_hi + 1] - str_off[s_lo] <= run_cap) ++s_hi;
    const int64_t nb = str_off[s_hi] - str_off[s_lo];
    if (nb > h->max_launch)  // (only a run of one string can be over run_cap)
      return fail(SW_ERR_ARG, "sw_encode_batch: a single string exceeds the launch limit");
    runs.emplace_back(s_lo, s_hi);
    max_b = std::max(max_b, nb);
    max_s = std::max(max_s, s_hi - s_lo);
    if (sp.dev) {
      max_sp = std::max(max_sp, nb / h->spt_min_len + 1);  // (the finder's capacity for the run)
    } else if (sp.n > 0) {
      int64_t j0, j1;
      sp_range(sp, str_off[s_lo] - str_off[0], str_off[s_hi] - str_off[0], &j0, &j1);
      max_sp = std::max(max_sp, j1 - j0);
    }
    s_lo = s_hi;
  }
  DeviceGuard g(h->device);
  if (!h->s_h2d) HIP_TRY(hipStreamCreateWithFlags(&h->s_h2d, hipStreamNonBlocking));
  if (!h->s_d2h) HIP_TRY(hipStreamCreateWithFlags(&h->s_d2h, hipStreamNonBlocking));
  if (!h->pool) h->pool = new sw::HostPool((int)std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
  const int64_t max_w = (max_b + 63) / 64 + 1;
  for (int slot = 0; slot < h->pipe_depth; ++slot) {
    auto& p = h->pipe[slot];
    if (sp.n > 0 && (p.cap_sp < max_sp || (!sp.dev && !p.h_sp))) {
      (void)hipHostFree(p.h_sp); (void)hipFree(p.d_sp);
      p.h_sp = nullptr; p.d_sp = nullptr; p.cap_sp = 0;
      // (pinned staging only for occurrences found on the host: the device finder writes d_sp itself)
      if (!sp.dev) HIP_TRY(hipHostMalloc(&p.h_sp, 3 * sizeof(int64_t) * max_sp, hipHostMallocDefault));
      HIP_TRY(hipMalloc(&p.d_sp, 3 * sizeof(int64_t) * max_sp));
      p.cap_sp = max_sp;
    }
    if (p.cap_bytes >= max_b && p.cap_str >= max_s) continue;
    const int64_t cb = std::max(max_b, p.cap_bytes), cs = std::max(max_s, p.cap_str), cw = (cb + 63) / 64 + 1;
    (void)hipHostFree(p.h_in); (void)hipHostFree(p.h_off); (void)hipHostFree(p.h_bits); (void)hipHostFree(p.h_out);
    (void)hipHostFree(p.h_oo); (void)hipHostFree(p.h_ntok);
    (void)hipFree(p.d_in); (void)hipFree(p.d_off); (void)hipFree(p.d_bits); (void)hipFree(p.d_out); (void)hipFree(p.d_oo);
    (void)hipFree(p.d_out16); (void)hipFree(p.d_ntok);
    p.cap_bytes = p.cap_str = 0;
    HIP_TRY(hipHostMalloc(&p.h_in, cb + 16, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&p.h_off, sizeof(int64_t) * (cs + 1), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&p.h_bits, sizeof(uint64_t) * cw, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&p.h_out, sizeof(int32_t) * cb, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&p.h_oo, sizeof(int64_t) * (cs + 1), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&p.h_ntok, sizeof(int64_t), hipHostMallocDefault));
    HIP_TRY(hipMalloc(&p.d_in, cb + 16));
    HIP_TRY(hipMalloc(&p.d_off, sizeof(int64_t) * (cs + 1)));
    HIP_TRY(hipMalloc(&p.d_bits, sizeof(uint64_t) * cw));
    HIP_TRY(hipMalloc(&p.d_out, sizeof(int32_t) * cb));
    HIP_TRY(hipMalloc(&p.d_oo, sizeof(int64_t) * (cs + 1)));
    HIP_TRY(hipMalloc(&p.d_out16, sizeof(uint16_t) * cb));
    HIP_TRY(hipMalloc(&p.d_ntok, sizeof(int64_t)));
    if (!p.e_in) HIP_TRY(hipEventCreateWithFlags(&p.e_in, hipEventDisableTiming));
    if (!p.e_comp) HIP_TRY(hipEventCreateWithFlags(&p.e_comp, hipEventDisableTiming));
    if (!p.e_out) HIP_TRY(hipEventCreateWithFlags(&p.e_out, hipEventDisableTiming));
    p.cap_bytes = cb;
    p.cap_str = cs;
  }
  (void)max_w;
  int32_t rc = ensure_workspace(h, max_b);
  if (rc) return rc;
  // caller ranges pinned by sw_encoder_pin_host: the input read over PCIe by the copy kernel (no
  // staging memcpy), the ids and offsets written by the device into the caller's arrays (no copy
  // or widening on the host)
  const uint8_t* in_dev =
      h->pipe_kcopy ? (const uint8_t*)h->pinned_dev(bytes + b0, std::max<int64_t>(str_off[n_str] - b0, 1)) : nullptr;
  int32_t* out_dev = h->pipe_kcopy ? (int32_t*)h->pinned_dev(out_ids, (int64_t)sizeof(int32_t) * out_cap) : nullptr;
  int64_t* oo_dev = h->pipe_kcopy ? (int64_t*)h->pinned_dev(out_off, (int64_t)sizeof(int64_t) * (n_str + 1)) : nullptr;
  const bool direct_out = out_dev && oo_dev;
  if (direct_out) {
    if (!h->d_done) HIP_TRY(hipMalloc(&h->d_done, 2 * sizeof(int64_t)));
    HIP_TRY(hipMemsetAsync(h->d_done, 0, 2 * sizeof(int64_t), h->s_d2h));
  }
  const bool count = stats && !chunk_bits;
  if (count) HIP_TRY(hipMemsetAsync(h->d_pcount, 0, sizeof(unsigned long long), h->stream));
  const bool was_timing = h->timing;
  const size_t was_used = h->ev_used, was_cls = h->ev_cls_used;
  h->timing = true;
  h->ev_used = 0;
  h->ev_cls_used = 0;
  auto restore = [&]() {
    h->timing = was_timing;
    h->ev_used = was_timing ? was_used : 0;
    h->ev_cls_used = was_timing ? was_cls : 0;
  };
  sw::HostPool& pool = *h->pool;
  double ms_stage = 0, ms_drain = 0;
  int64_t done = 0;
  int64_t p_nsp[4] = {0, 0, 0, 0};  // special-token occurrences staged per slot
  static const bool trace = std::getenv("SW_PIPE_TRACE") != nullptr;  // (diagnostic timeline)
  auto stamp = [&](const char* what, size_t k) {
    if (trace)
      std::fprintf(stderr, "pipe %8.3f %-10s %zu\n",
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count(), what, k);
  };
  auto stage = [&](size_t k) -> int32_t {
    auto& p = h->pipe[k % h->pipe_depth];
    const int64_t s_lo = runs[k].first, s_hi = runs[k].second, a0 = str_off[s_lo], nb = str_off[s_hi] - a0;
    auto t = std::chrono::steady_clock::now();
    const uint8_t* src = bytes + a0;
    if (!in_dev)
      pool.parallel_for(nb, [&](int64_t lo, int64_t hi) { std::memcpy(p.h_in + lo, src + lo, (size_t)(hi - lo)); });
    for (int64_t j = 0; j <= s_hi - s_lo; ++j) p.h_off[j] = str_off[s_lo + j] - a0;
    if (sp.dev) {
      p_nsp[k % h->pipe_depth] = nb / h->spt_min_len + 1;  // (found on the device after the upload)
    } else if (sp.n > 0) {  // the run's special-token occurrences, rebased: positions, then lengths and ids (int32)
      int64_t j0, j1;
      sp_range(sp, a0 - b0, a0 - b0 + nb, &j0, &j1);
      const int64_t m = j1 - j0;
      int32_t* l32 = (int32_t*)(p.h_sp + m);
      for (int64_t j = 0; j < m; ++j) {
        p.h_sp[j] = sp.pos[j0 + j] - (a0 - b0);
        l32[j] = sp.len[j0 + j];
        l32[m + j] = sp.id[j0 + j];
      }
      p_nsp[k % h->pipe_depth] = m;
    }
    if (chunk_bits) {  // the run's bits, realigned to its first byte
      const int64_t g0 = a0 - b0, nw = (nb + 63) / 64, last_q = (str_off[n_str] - b0 - 1) / 64;
      pool.parallel_for(nw, [&](int64_t lo, int64_t hi) {
        for (int64_t w = lo; w < hi; ++w) {
          const int64_t bit = g0 + 64 * w, q = bit >> 6, r = bit & 63;
          uint64_t x = chunk_bits[q] >> r;
          if (r && q + 1 <= last_q) x |= chunk_bits[q + 1] << (64 - r);
          p.h_bits[w] = x;
        }
      });
    }
    ms_stage += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    stamp("staged", k);
    return SW_OK;
  };
  auto issue = [&](size_t k) -> int32_t {
    auto& p = h->pipe[k % h->pipe_depth];
    const int64_t s_lo = runs[k].first, s_hi = runs[k].second, nb = str_off[s_hi] - str_off[s_lo], ns = s_hi - s_lo;
    const int64_t n_bits = chunk_bits ? (int64_t)sizeof(uint64_t) * ((nb + 63) / 64) : 0;
    const int64_t m_sp = sp.n > 0 ? p_nsp[k % h->pipe_depth] : 0, n_sp_bytes = sp.dev ? 0 : 16 * m_sp;  // (8 + 4 + 4 B each)
    if (h->pipe_kcopy) {
      const uint8_t* in_src = in_dev ? in_dev + (str_off[s_lo] - b0) : p.h_in;
      const CopySegs c{{in_src, (const uint8_t*)p.h_off, (const uint8_t*)p.h_bits, (const uint8_t*)p.h_sp, nullptr, nullptr},
                       {p.d_in, (uint8_t*)p.d_off, (uint8_t*)p.d_bits, (uint8_t*)p.d_sp, nullptr, nullptr},
                       {nb, (int64_t)sizeof(int64_t) * (ns + 1), n_bits, n_sp_bytes, 0, 0}};
      hipLaunchKernelGGL(k_copy_segs, dim3(128), dim3(256), 0, h->s_h2d, c);
      HIP_TRY(hipGetLastError());
    } else {
      HIP_TRY(hipMemcpyAsync(p.d_in, p.h_in, (size_t)nb, hipMemcpyHostToDevice, h->s_h2d));
      HIP_TRY(hipMemcpyAsync(p.d_off, p.h_off, sizeof(int64_t) * (ns + 1), hipMemcpyHostToDevice, h->s_h2d));
      if (chunk_bits) HIP_TRY(hipMemcpyAsync(p.d_bits, p.h_bits, (size_t)n_bits, hipMemcpyHostToDevice, h->s_h2d));
      if (n_sp_bytes > 0) HIP_TRY(hipMemcpyAsync(p.d_sp, p.h_sp, (size_t)n_sp_bytes, hipMemcpyHostToDevice, h->s_h2d));
    }
    HIP_TRY(hipEventRecord(p.e_in, h->s_h2d));
    HIP_TRY(hipStreamWaitEvent(h->stream, p.e_in, 0));
    DevSpecials dsp;
    if (m_sp > 0) {
      dsp.pos = p.d_sp; dsp.len = (const int32_t*)(p.d_sp + m_sp); dsp.id = dsp.len + m_sp; dsp.n = m_sp;
    }
    if (sp.dev) {  // the occurrences found on the device, the count left there (p.d_sp's tail)
      int64_t* d_cnt = p.d_sp + 2 * m_sp;
      const int32_t r = find_specials_device(h, p.d_in, nb, p.d_off, ns, p.d_sp, (int32_t*)dsp.len, (int32_t*)dsp.id,
                                             m_sp, d_cnt, h->stream);
      if (r) return r;
      dsp.n_dev = d_cnt;
    }
    const int32_t r = encode_device(h, p.d_in, nb, p.d_off, ns, chunk_bits ? p.d_bits : nullptr, dsp, p.d_out, false,
                                    p.d_oo, h->stream, nullptr, pattern);
    if (r) return r;
    if (count && nb > 0)
      hipLaunchKernelGGL(k_popcount, dim3(1024), dim3(256), 0, h->stream, h->d_pbits, (nb + 63) / 64, h->d_pcount);
    if (h->pipe_kcopy) {
      // the download kernel runs on s_d2h beside the next run's encode, which rewrites d_total
      HIP_TRY(hipMemcpyAsync(p.d_ntok, h->d_total, sizeof(int64_t), hipMemcpyDeviceToDevice, h->stream));
    } else if (narrow) {
      hipLaunchKernelGGL(k_pack16, dim3(2048), dim3(256), 0, h->stream, p.d_out, h->d_total, p.d_out16);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(p.h_ntok, h->d_total, sizeof(int64_t), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipEventRecord(p.e_comp, h->stream));
    if (h->pipe_kcopy) {
      HIP_TRY(hipStreamWaitEvent(h->s_d2h, p.e_comp, 0));
      if (direct_out) {
        hipLaunchKernelGGL(k_push_direct, dim3(128), dim3(256), 0, h->s_d2h, p.d_out, p.d_ntok, p.d_oo, ns + 1, out_dev,
                           oo_dev + s_lo, out_cap, h->d_done);
        hipLaunchKernelGGL(k_push_advance, dim3(1), dim3(64), 0, h->s_d2h, p.d_ntok, out_cap, h->d_done);
      } else {
        hipLaunchKernelGGL(k_push_run, dim3(128), dim3(256), 0, h->s_d2h, p.d_out, p.d_ntok, narrow ? 0 : 1,
                           p.h_out, p.d_oo, ns + 1, p.h_oo);
      }
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(p.e_out, h->s_d2h));
    }
    return SW_OK;
  };
  auto drain = [&](size_t k) -> int32_t {
    auto& p = h->pipe[k % h->pipe_depth];
    const int64_t s_lo = runs[k].first, s_hi = runs[k].second, ns = s_hi - s_lo;
    HIP_TRY(hipEventSynchronize(p.e_comp));
    stamp("encoded", k);
    const int64_t nt = *p.h_ntok;
    if (done + nt > out_cap) return fail(SW_ERR_CAP, "sw_encode_batch: out_cap too small");
    auto t = std::chrono::steady_clock::now();
    if (!h->pipe_kcopy) {
      HIP_TRY(hipStreamWaitEvent(h->s_d2h, p.e_comp, 0));
      if (nt > 0)
        HIP_TRY(hipMemcpyAsync(p.h_out, narrow ? (void*)p.d_out16 : (void*)p.d_out,
                               (size_t)nt * (narrow ? 2 : 4), hipMemcpyDeviceToHost, h->s_d2h));
      HIP_TRY(hipMemcpyAsync(p.h_oo, p.d_oo, sizeof(int64_t) * (ns + 1), hipMemcpyDeviceToHost, h->s_d2h));
      HIP_TRY(hipEventRecord(p.e_out, h->s_d2h));
    }
    HIP_TRY(hipEventSynchronize(p.e_out));
    stamp("pushed", k);
    if (direct_out) {  // (the device wrote them into the caller's arrays)
      done += nt;
      ms_drain += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
      return SW_OK;
    }
    int32_t* dst = out_ids + done;
    if (narrow) {
      const uint16_t* s16 = (const uint16_t*)p.h_out;
      pool.parallel_for(nt, [&](int64_t lo, int64_t hi) { widen16_stream(s16 + lo, dst + lo, hi - lo); });
    } else {
      const int32_t* s32 = (const int32_t*)p.h_out;
      pool.parallel_for(nt, [&](int64_t lo, int64_t hi) { std::memcpy(dst + lo, s32 + lo, sizeof(int32_t) * (hi - lo)); });
    }
    for (int64_t j = 0; j <= ns; ++j) out_off[s_lo + j] = p.h_oo[j] + done;
    done += nt;
    stamp("drained", k);
    ms_drain += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    return SW_OK;
  };
  // host order: stage k, issue k, then drain the oldest run when every slot is taken (pipe_depth
  // runs in flight: run k's upload overlaps the encodes and downloads of the runs before it)
  auto bail = [&](int32_t r) {  // leave nothing in flight on the slots' buffers
    (void)hipStreamSynchronize(h->s_h2d);
    (void)hipStreamSynchronize(h->stream);
    (void)hipStreamSynchronize(h->s_d2h);
    restore();
    return r;
  };
  const size_t depth = (size_t)h->pipe_depth;
  size_t next_drain = 0;
  for (size_t k = 0; k < runs.size(); ++k) {
    rc = stage(k);
    if (!rc) rc = issue(k);
    if (!rc && next_drain + depth <= k + 1) rc = drain(next_drain++);  // frees run k + 1's slot
    if (rc) return bail(rc);
  }
  while (next_drain < runs.size())
    if ((rc = drain(next_drain++))) return bail(rc);
  if (n_str == 0) out_off[0] = 0;
  const double k_ms = sw_encoder_last_kernel_ms(h) * (double)runs.size();
  int64_t n_chunks = -1;
  if (count) {
    unsigned long long c = 0;
    HIP_TRY(hipMemcpy(&c, h->d_pcount, sizeof(c), hipMemcpyDeviceToHost));
    n_chunks = (int64_t)c;
  }
  restore();
  if (stats) {
    stats->n_bytes = str_off[n_str] - b0;
    stats->n_chunks = n_chunks;
    stats->n_tokens = done;
    stats->ms_presplit = 0;
    stats->ms_h2d = ms_stage;   // (host staging into pinned memory; the uploads overlap)
    stats->ms_kernels = k_ms;
    stats->ms_d2h = ms_drain;   // (downloads + copies out, overlapped with the next run's encode)
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
  }
  return SW_OK;
}

}  // namespace

namespace {

// sw_encode_batch(_ex) with the batch's special-token occurrences found (sp, relative to str_off[0])
int32_t encode_batch_impl(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str, int32_t pattern,
                          const uint64_t* chunk_bits, const HostSpecials& sp, int32_t* out_ids, int64_t out_cap,
                          int64_t* out_off, sw_stats* stats) {
  auto T0 = std::chrono::steady_clock::now();
  if (!h || !str_off || !out_off || n_str < 0) return fail(SW_ERR_ARG, "sw_encode_batch: bad arguments");
  const int64_t b0 = n_str > 0 ? str_off[0] : 0;
  const int64_t n_bytes = n_str > 0 ? str_off[n_str] - b0 : 0;
  if (n_bytes < 0 || (n_bytes > 0 && !bytes)) return fail(SW_ERR_ARG, "sw_encode_batch: bad string offsets");
  for (int64_t s = 0; s < n_str; ++s)
    if (str_off[s + 1] < str_off[s]) return fail(SW_ERR_ARG, "sw_encode_batch: string offsets not monotone");
  if (n_bytes > 0 && !out_ids) return fail(SW_ERR_ARG, "sw_encode_batch: null out_ids");
  if (!chunk_bits && pattern != SW_PAT_CL100K && pattern != SW_PAT_GPT2 && pattern != SW_PAT_NONE)
    return fail(SW_ERR_ARG, "sw_encode_batch: bad pattern");
  if (h->pipe_run > 0 && n_bytes > 2 * h->pipe_run && !(h->host_presplit && !chunk_bits))
    return encode_batch_pipelined(h, bytes, str_off, n_str, pattern, chunk_bits, sp, out_ids, out_cap, out_off, stats,
                                  T0);
  if (n_bytes > h->max_launch) {
    // one device launch addresses < 2^30 bytes: encode runs of whole strings separately
    int64_t done = 0, s_lo = 0;
    if (stats) *stats = sw_stats{};
    while (s_lo < n_str) {
      int64_t s_hi = s_lo + 1;
      while (s_hi < n_str && str_off[s_hi + 1] - str_off[s_lo] <= h->max_launch) ++s_hi;
      if (str_off[s_hi] - str_off[s_lo] > h->max_launch)
        return fail(SW_ERR_ARG, "sw_encode_batch: a single string exceeds the launch limit (2^30 - 64 bytes)");
      std::vector<uint64_t> sub;
      if (chunk_bits) {  // the run's bits, realigned to its first byte
        const int64_t g0 = str_off[s_lo] - b0, nb = str_off[s_hi] - str_off[s_lo];
        sub.assign((size_t)((nb + 63) / 64 + 1), 0ULL);
        for (int64_t w = 0; w < (nb + 63) / 64; ++w) {
          const int64_t bit = g0 + 64 * w, q = bit >> 6, r = bit & 63;
          uint64_t x = chunk_bits[q] >> r;
          if (r && q + 1 <= (str_off[n_str] - b0 - 1) / 64) x |= chunk_bits[q + 1] << (64 - r);
          sub[(size_t)w] = x;
        }
      }
      sw_stats st{};
      HostSpecials ssp = sp;  // (the run's occurrences, rebased to its first byte)
      int64_t j0 = 0, j1 = 0;
      std::vector<int64_t> spos;
      if (sp.n > 0 && !sp.dev) {
        const int64_t g0 = str_off[s_lo] - b0;
        sp_range(sp, g0, str_off[s_hi] - b0, &j0, &j1);
        spos.resize((size_t)(j1 - j0));
        for (int64_t j = j0; j < j1; ++j) spos[(size_t)(j - j0)] = sp.pos[j] - g0;
        ssp.pos = spos.data(); ssp.len = sp.len + j0; ssp.id = sp.id + j0; ssp.n = j1 - j0;
      }
      int32_t rc = encode_batch_impl(h, bytes, str_off + s_lo, s_hi - s_lo, pattern, chunk_bits ? sub.data() : nullptr,
                                     ssp, out_ids + done, out_cap - done, out_off + s_lo, &st);
      if (rc) return rc;
      for (int64_t s = s_lo; s <= s_hi; ++s) out_off[s] += done;
      done = out_off[s_hi];
      if (stats) {
        // (a run without a chunk count -- caller bits -- makes the total unknown: -1)
        stats->n_chunks = (stats->n_chunks < 0 || st.n_chunks < 0) ? -1 : stats->n_chunks + st.n_chunks;
        stats->n_bytes += st.n_bytes; stats->n_tokens += st.n_tokens;
        stats->ms_presplit += st.ms_presplit; stats->ms_h2d += st.ms_h2d; stats->ms_kernels += st.ms_kernels;
        stats->ms_d2h += st.ms_d2h;
      }
      s_lo = s_hi;
    }
    if (stats)
      stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
    return SW_OK;
  }
  const int64_t n_words = (n_bytes + 63) / 64;
  std::vector<uint64_t> own_bits;
  double ms_pre = 0;
  int64_t n_chunks = -1;
  const bool device_presplit = !chunk_bits && !h->host_presplit;
  if (!chunk_bits && !device_presplit) {
    own_bits.resize((size_t)std::max<int64_t>(n_words, 1));
    auto a = std::chrono::steady_clock::now();
    n_chunks = sp.n > 0 ? sw_presplit_host_specials(bytes, str_off, n_str, pattern, sp.pos, sp.len, sp.n, own_bits.data(), 0)
                        : sw_presplit_host(bytes, str_off, n_str, pattern, own_bits.data(), 0);
    if (n_chunks < 0) return fail((int32_t)n_chunks, "sw_encode_batch: bad pattern or offsets");
    ms_pre = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    chunk_bits = own_bits.data();
  }
  DeviceGuard g(h->device);
  // device staging (grown on demand)
  if (n_bytes > h->io_bytes || n_str > h->io_str) {
    free_io(h);
    const int64_t nb = std::max<int64_t>(n_bytes, 1), ns = std::max<int64_t>(n_str, 1);
    HIP_TRY(hipMalloc(&h->d_bytes, nb));
    HIP_TRY(hipMalloc(&h->d_str_off, sizeof(int64_t) * (ns + 1)));
    HIP_TRY(hipMalloc(&h->d_bits, sizeof(uint64_t) * ((nb + 63) / 64)));
    HIP_TRY(hipMalloc(&h->d_out, sizeof(int32_t) * nb));
    HIP_TRY(hipMalloc(&h->d_out_off, sizeof(int64_t) * (ns + 1)));
    h->io_bytes = nb; h->io_str = ns;
  }
  const int64_t sp_need = sp.dev ? n_bytes / h->spt_min_len + 1 : sp.n;  // (the device finder's capacity)
  if (sp_need > h->sp_cap) {
    (void)hipFree(h->d_sp_pos); (void)hipFree(h->d_sp_len); (void)hipFree(h->d_sp_id);
    h->d_sp_pos = nullptr; h->d_sp_len = nullptr; h->d_sp_id = nullptr; h->sp_cap = 0;
    HIP_TRY(hipMalloc(&h->d_sp_pos, sizeof(int64_t) * sp_need));
    HIP_TRY(hipMalloc(&h->d_sp_len, sizeof(int32_t) * sp_need));
    HIP_TRY(hipMalloc(&h->d_sp_id, sizeof(int32_t) * sp_need));
    h->sp_cap = sp_need;
  }
  if (sp.dev && !h->d_nsp) HIP_TRY(hipMalloc(&h->d_nsp, sizeof(int64_t)));
  std::vector<int64_t> rel((size_t)n_str + 1);
  for (int64_t s = 0; s <= n_str; ++s) rel[s] = n_str > 0 ? str_off[s] - b0 : 0;
  auto a = std::chrono::steady_clock::now();
  hipStream_t st = h->stream;
  if (n_bytes > 0) {
    HIP_TRY(hipMemcpyAsync(h->d_bytes, bytes + b0, n_bytes, hipMemcpyHostToDevice, st));
    if (!device_presplit)
      HIP_TRY(hipMemcpyAsync(h->d_bits, chunk_bits, sizeof(uint64_t) * n_words, hipMemcpyHostToDevice, st));
  }
  HIP_TRY(hipMemcpyAsync(h->d_str_off, rel.data(), sizeof(int64_t) * (n_str + 1), hipMemcpyHostToDevice, st));
  DevSpecials dsp;
  if (sp.dev) {
    const int32_t r = find_specials_device(h, h->d_bytes, n_bytes, h->d_str_off, n_str, h->d_sp_pos, h->d_sp_len,
                                           h->d_sp_id, h->sp_cap, h->d_nsp, st);
    if (r) return r;
    dsp.pos = h->d_sp_pos; dsp.len = h->d_sp_len; dsp.id = h->d_sp_id; dsp.n = h->sp_cap; dsp.n_dev = h->d_nsp;
  } else if (sp.n > 0) {
    HIP_TRY(hipMemcpyAsync(h->d_sp_pos, sp.pos, sizeof(int64_t) * sp.n, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->d_sp_len, sp.len, sizeof(int32_t) * sp.n, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->d_sp_id, sp.id, sizeof(int32_t) * sp.n, hipMemcpyHostToDevice, st));
    dsp.pos = h->d_sp_pos; dsp.len = h->d_sp_len; dsp.id = h->d_sp_id; dsp.n = sp.n;
  }
  HIP_TRY(hipStreamSynchronize(st));
  double ms_h2d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  int64_t n_tok = 0;
  const bool was_timing = h->timing;
  const size_t was_used = h->ev_used, was_cls = h->ev_cls_used;
  h->timing = true;
  h->ev_used = 0;
  h->ev_cls_used = 0;
  int32_t rc = encode_device(h, h->d_bytes, n_bytes, h->d_str_off, n_str, device_presplit ? nullptr : h->d_bits, dsp,
                             h->d_out, false, h->d_out_off, st, &n_tok, pattern);
  if (rc == SW_OK && device_presplit && stats && n_bytes > 0) {  // chunk count for the stats
    HIP_TRY(hipMemsetAsync(h->d_pcount, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_popcount, dim3(1024), dim3(256), 0, st, h->d_pbits, n_words, h->d_pcount);
    unsigned long long c = 0;
    HIP_TRY(hipMemcpyAsync(&c, h->d_pcount, sizeof(c), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    n_chunks = (int64_t)c;
  }
  const double k_ms = sw_encoder_last_kernel_ms(h);
  h->timing = was_timing;
  h->ev_used = was_timing ? was_used : 0;
  h->ev_cls_used = was_timing ? was_cls : 0;
  if (rc) return rc;
  if (n_tok > out_cap) return fail(SW_ERR_CAP, "sw_encode_batch: out_cap too small");
  a = std::chrono::steady_clock::now();
  if (n_tok > 0) HIP_TRY(hipMemcpyAsync(out_ids, h->d_out, sizeof(int32_t) * n_tok, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(out_off, h->d_out_off, sizeof(int64_t) * (n_str + 1), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  double ms_d2h = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  if (stats) {
    stats->n_bytes = n_bytes;
    stats->n_chunks = n_chunks;
    stats->n_tokens = n_tok;
    stats->ms_presplit = ms_pre;
    stats->ms_h2d = ms_h2d;
    stats->ms_kernels = k_ms;
    stats->ms_d2h = ms_d2h;
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
  }
  return SW_OK;
}

}  // namespace

extern "C" int32_t sw_encode_batch(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                                   int32_t pattern, const uint64_t* chunk_bits, int32_t* out_ids, int64_t out_cap,
                                   int64_t* out_off, sw_stats* stats) {
  return encode_batch_impl(h, bytes, str_off, n_str, pattern, chunk_bits, HostSpecials{}, out_ids, out_cap, out_off,
                           stats);
}

// device memory the device special-token finder may take for sw_encode_batch_ex (its worst-case
// occurrence arrays of every pipeline slot and its per-tile lists); beyond it the host threads find them
constexpr int64_t kSpDeviceBudget = 1LL << 30;

extern "C" int32_t sw_encode_batch_ex(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                                      int32_t pattern, const uint64_t* chunk_bits, const sw_specials* specials,
                                      int32_t* out_ids, int64_t out_cap, int64_t* out_off, sw_stats* stats) {
  if (!specials || specials->n == 0)
    return encode_batch_impl(h, bytes, str_off, n_str, pattern, chunk_bits, HostSpecials{}, out_ids, out_cap, out_off,
                             stats);
  if (!h || !str_off || n_str < 0) return fail(SW_ERR_ARG, "sw_encode_batch_ex: bad arguments");
  for (int64_t k = 0; k < specials->n; ++k)
    if (specials->ids && (specials->ids[k] < 0 || specials->ids[k] == INT32_MAX))
      return fail(SW_ERR_ARG, "sw_encode_batch_ex: special token ids must be in [0, 2^31 - 2]");
  // the device finder: every special <= 64 bytes, the device pre-split (the host pre-split needs the
  // occurrences on the host), and room for its worst case (n / shortest special occurrences)
  if (h->device_specials && !chunk_bits && !h->host_presplit) {
    int32_t rc = set_specials(h, specials);
    if (rc) return rc;
    const int64_t nb = n_str > 0 ? str_off[n_str] - str_off[0] : 0;
    const int64_t run = h->pipe_run > 0 && nb > 2 * h->pipe_run ? std::min(h->pipe_run, h->max_launch)
                                                                   : std::min(nb, h->max_launch);
    // (the finder sizes its arrays for the worst case -- every run packed with the shortest special:
    // 24 B per possible occurrence and slot, and each tile's list -- so short specials on large runs
    // fall back to the host threads rather than take gigabytes of device memory)
    const int64_t slots = h->pipe_run > 0 && nb > 2 * h->pipe_run ? h->pipe_depth : 1;
    const int64_t worst = 24 * (run / h->spt_min_len + 1) * slots +
                          4 * ((run + kTile - 1) / kTile) * (kTile / h->spt_min_len + 1);
    if (h->spt_dev && worst <= kSpDeviceBudget && 16 * (run / h->spt_min_len + 1) <= (int64_t)1 << 31) {
      HostSpecials sp;
      sp.dev = true;
      sp.n = 1;
      for (int64_t k = 0; k < specials->n; ++k)
        if (specials->ids[k] > 0xFFFD) sp.narrow = false;
      return encode_batch_impl(h, bytes, str_off, n_str, pattern, chunk_bits, sp, out_ids, out_cap, out_off, stats);
    }
  }
  const int64_t cnt = sw_find_specials_host(bytes, str_off, n_str, specials, nullptr, nullptr, nullptr, 0, 0);
  if (cnt < 0) return fail((int32_t)cnt, "sw_encode_batch_ex: bad special tokens or string offsets");
  std::vector<int64_t> pos((size_t)std::max<int64_t>(cnt, 1));
  std::vector<int32_t> len(pos.size()), id(pos.size());
  if (cnt > 0) {
    const int64_t got = sw_find_specials_host(bytes, str_off, n_str, specials, pos.data(), len.data(), id.data(), cnt, 0);
    if (got != cnt) return fail(SW_ERR_ARG, "sw_encode_batch_ex: special-token scan");
  }
  HostSpecials sp;
  sp.pos = pos.data(); sp.len = len.data(); sp.id = id.data(); sp.n = cnt;
  for (int64_t k = 0; k < cnt; ++k)
    if (id[(size_t)k] > 0xFFFD) sp.narrow = false;
  return encode_batch_impl(h, bytes, str_off, n_str, pattern, chunk_bits, sp, out_ids, out_cap, out_off, stats);
}

extern "C" int32_t sw_encoder_last_counts(sw_encoder* h, int64_t* out4) {
  if (!h || !out4) return fail(SW_ERR_ARG, "sw_encoder_last_counts: bad arguments");
  DeviceGuard g(h->device);
  for (int i = 0; i < 4; ++i) out4[i] = 0;
  out4[3] = h->last_tiles;
  if (!h->ws_pending || h->last_tiles == 0) return SW_OK;
  HIP_TRY(hipEventSynchronize(h->ws_done));
  std::vector<uint32_t> slots((size_t)h->last_tiles), nref((size_t)h->last_tiles);
  HIP_TRY(hipMemcpy(slots.data(), h->d_tile_slots, sizeof(uint32_t) * slots.size(), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(nref.data(), h->d_tile_nref, sizeof(uint32_t) * nref.size(), hipMemcpyDeviceToHost));
  int64_t q = 0;
  HIP_TRY(hipMemcpy(&q, h->d_qtotal, sizeof(q), hipMemcpyDeviceToHost));
  for (size_t t = 0; t < slots.size(); ++t) { out4[0] += slots[t]; out4[1] += nref[t]; }
  out4[2] = q;
  return SW_OK;
}

extern "C" int32_t sw_presplit_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                                      int64_t n_str, int32_t pattern, uint64_t* d_chunk_bits, void* stream,
                                      int64_t* n_chunks_host) {
  if (!h || n_bytes < 0 || n_str < 0 || !d_str_off || (n_bytes > 0 && (!d_bytes || !d_chunk_bits)))
    return fail(SW_ERR_ARG, "sw_presplit_device: bad arguments");
  if (pattern != SW_PAT_CL100K && pattern != SW_PAT_GPT2 && pattern != SW_PAT_NONE)
    return fail(SW_ERR_ARG, "sw_presplit_device: bad pattern");
  DeviceGuard g(h->device);
  hipStream_t st = (hipStream_t)stream;  // (NULL: the null stream, as torch's default stream)
  int32_t rc = ensure_workspace(h, n_bytes);
  if (rc) return rc;
  if (n_bytes > 0)
    hipLaunchKernelGGL(k_tile_strings, dim3((unsigned)(((n_bytes + kTile - 1) / kTile + 255) / 256)), dim3(256), 0, st,
                       d_str_off, n_str, (n_bytes + kTile - 1) / kTile, h->d_tile_slo, nullptr);
  HIP_TRY(launch_presplit(st, d_bytes, n_bytes, d_str_off, n_str, pattern, d_chunk_bits, h->d_tile_slo));
  if (n_chunks_host) {
    *n_chunks_host = 0;
    if (n_bytes > 0) {
      HIP_TRY(hipMemsetAsync(h->d_pcount, 0, sizeof(unsigned long long), st));
      hipLaunchKernelGGL(k_popcount, dim3(1024), dim3(256), 0, st, d_chunk_bits, (n_bytes + 63) / 64, h->d_pcount);
      unsigned long long c = 0;
      HIP_TRY(hipMemcpyAsync(&c, h->d_pcount, sizeof(c), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      *n_chunks_host = (int64_t)c;
    }
  }
  return SW_OK;
}
