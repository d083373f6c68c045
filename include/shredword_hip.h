/* shredword_hip.h -- C-ABI of the MI355X-native BPE encode path.
 *
 * This is the drop-in boundary under shredword's Python tokenizer surface.  The reference
 * binds its native code through ctypes (`shredword/cbase.py:5-59`: library discovery,
 * `ctypes.CDLL`, per-function argtypes/restype, opaque `Trainer*` handle, int status codes
 * mapped to Python exceptions in `shredword/trainer.py:14-25`).  The reference has no native
 * encode: `BaseTokenizer.encode` is abstract (`shredword/base.py:108`) and its semantics are
 * pinned by the primitives `get_stats` (base.py:10-20), `merge` (base.py:22-36) and
 * `apply_regex` (base.py:38-58).  Each entry point below names the reference interface whose
 * role it takes.
 *
 * Conventions
 *   - Plain pointers and sizes; no torch types.  Status: SW_OK (0) or a negative SW_ERR_*.
 *     Never exit(): the reference's `exit(EXIT_FAILURE)` paths (bpe.cpp:113-121) are replaced
 *     by status codes plus sw_last_error() (thread-local message).
 *   - The caller owns every buffer it passes.  The encoder handle owns its device copy of the
 *     merge table, its workspace and its stream.
 *   - One handle per host thread (a handle is not internally locked).  The device workspace
 *     belongs to the handle: a launch on a stream other than the previous launch's waits for
 *     that launch (a HIP event), so calls on one handle are ordered whatever their streams.
 *   - Ids are int32.  Vocab ids 0..255 are raw bytes (base.py:74); a merge value is both the
 *     pair's rank and the new token id (base.py:137,147).
 */
#ifndef SHREDWORD_HIP_H
#define SHREDWORD_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SW_OK 0
#define SW_ERR_ARG (-1)     /* bad argument (null pointer, negative size, bad table) */
#define SW_ERR_HIP (-2)     /* HIP runtime error (message has the HIP error string) */
#define SW_ERR_ALLOC (-3)   /* host or device allocation failed */
#define SW_ERR_CAP (-4)     /* output capacity too small */
#define SW_ERR_NODEV (-5)   /* no usable gfx950 device */

/* Pre-split patterns.  CL100K is the pattern apply_regex hard-codes (base.py:56); GPT2 is the
 * alternative quoted in its docstring (base.py:46); NONE encodes each string as one chunk. */
#define SW_PAT_CL100K 0
#define SW_PAT_GPT2 1
#define SW_PAT_NONE 2

/* Synthetic corpus kinds (bench configs) */
#define SW_CORPUS_ASCII 0
#define SW_CORPUS_MIXED 1
#define SW_CORPUS_STRESS 2
#define SW_CORPUS_ENTROPY 3   /* low repetition: a flat Zipf over 1 M words in six scripts */

typedef struct sw_encoder sw_encoder;

typedef struct sw_stats {
  int64_t n_bytes;      /* input bytes */
  int64_t n_chunks;     /* pre-split chunks */
  int64_t n_tokens;     /* output ids */
  double ms_presplit;   /* host pre-split (0 if the caller supplied chunk_bits) */
  double ms_h2d;        /* host->device copies */
  double ms_kernels;    /* device time of the encode kernels (HIP events) */
  double ms_d2h;        /* device->host copies */
  double ms_total;      /* wall time of the call */
} sw_stats;

/* Last error message of this thread ("" if none).  Replaces the reference's stderr+exit. */
const char* sw_last_error(void);

/* Library / build identification, e.g. "shredword_hip 0.1 gfx950". */
const char* sw_version(void);

/* Number of visible HIP devices (0 if none / no runtime).  Never fails. */
int32_t sw_device_count(void);

/* ---- encoder lifecycle (role of create_trainer / bpe_trainer_destroy, bpe.h:62-64) ----
 * pairs: n x 2 int32 (a, b); vals: n int32, the value merges[(a, b)] (rank == new id).
 * Duplicate pairs: the LAST occurrence wins, as dict assignment does (base.py:145-148).
 * Values must be in [0, 2^31-1].  device: HIP device ordinal. */
int32_t sw_encoder_create(const int32_t* pairs, const int32_t* vals, int64_t n, int32_t device,
                          sw_encoder** out);
void sw_encoder_destroy(sw_encoder* h);

/* Pre-allocate the device workspace for inputs up to max_bytes / max_strings (optional;
 * encode grows it on demand otherwise). */
int32_t sw_encoder_reserve(sw_encoder* h, int64_t max_bytes, int64_t max_strings);

/* Pin (page-lock and map for the device) a caller's host buffer that it passes to sw_encode_batch
 * call after call (no reference counterpart: the reference has no device path).  A batch whose
 * input bytes lie inside a pinned range is read straight over PCIe (no staging copy on the host);
 * a batch whose out_ids [out_cap] and out_off [n_str + 1] both lie inside pinned ranges gets its
 * ids (int32) and string offsets written there by the device (no copy or widening pass on the
 * host).  Results are the same either way.  A range stays pinned until sw_encoder_unpin_host(ptr)
 * or sw_encoder_destroy; the caller keeps it alive that long.  SW_ERR_HIP if the runtime refuses
 * the range, SW_ERR_ARG for an unknown ptr. */
int32_t sw_encoder_pin_host(sw_encoder* h, void* ptr, int64_t bytes);
int32_t sw_encoder_unpin_host(sw_encoder* h, void* ptr);

/* Encoder options (sw_encoder_set_option).  Every option leaves the results unchanged.
 *   SW_OPT_PATTERN         pre-split pattern (SW_PAT_*) sw_encode_device uses when it is given
 *                          no chunk bitmap (default SW_PAT_CL100K)
 *   SW_OPT_HOST_PRESPLIT   1: sw_encode_batch without a bitmap pre-splits on the host threads
 *                          (sw_presplit_host) instead of on the device (default 0) */
#define SW_OPT_PATTERN 5
#define SW_OPT_HOST_PRESPLIT 6
/*   SW_OPT_MAX_LAUNCH_BYTES  sw_encode_batch encodes larger batches as several launches of
 *                          whole strings (0 = the 2^30 - 64 byte device limit; any value >= 64:
 *                          a smaller device workspace) */
#define SW_OPT_MAX_LAUNCH_BYTES 8
/*   SW_OPT_PIPE_RUN_BYTES  sw_encode_batch of more than 2 runs of this many bytes (default 128 MiB; 0:
 *                          never) pipelines runs of whole strings: pinned staging copied by a pool of
 *                          host threads, uploads, encodes and downloads of consecutive runs
 *                          overlapping, ids downloaded as 16 bits when every id fits
 *   SW_OPT_PIPE_DEPTH      runs in flight in that pipeline, 2 .. 4 (default 3) */
#define SW_OPT_PIPE_RUN_BYTES 9
#define SW_OPT_PIPE_DEPTH 12
/*   SW_OPT_DEVICE_SPECIALS 1 (default): sw_encode_batch_ex finds the special-token occurrences on the
 *                          device (sw_find_specials_device, launch by launch) when every special is
 *                          <= 64 bytes and the pre-split is the device's; 0: on the host threads. */
#define SW_OPT_DEVICE_SPECIALS 18
/* (Options 1-4, 7, 10, 11, 13, 14, 17 and 19 are the library's measurement and test switches --
 * the memoisation shortcuts, the dedupe table's limits, the alternative kernels -- documented in
 * shredword_amd/csrc/test_options.h, not part of this interface.  Option 15 (a round-2 A/B knob)
 * and 16 (replaced by sw_encode_ex.out_bits) are rejected.) */
int32_t sw_encoder_set_option(sw_encoder* h, int32_t option, int64_t value);

/* Encoder facts (sw_encoder_get_info): distinct merges, whole-chunk table entries, whether the
 * pair table uses the wide (>16-bit ids) layout, whether kernels run on 16-bit ids. */
#define SW_INFO_MERGES 1
#define SW_INFO_CHUNK_ENTRIES 2
#define SW_INFO_WIDE_TABLE 3
#define SW_INFO_IDS16 4
#define SW_INFO_SPLIT 5     /* the table is well-formed: long chunks may take the split path */
#define SW_INFO_DEDUPE_SLOTS 6  /* entries of the dedupe table now (it grows after a launch overflows it) */
#define SW_INFO_CHUNK_TABLE_BYTES 7  /* device bytes of the whole-chunk table (its 64-byte lines) */
int64_t sw_encoder_get_info(const sw_encoder* h, int32_t what);

/* ---- host pre-split (apply_regex, base.py:38-58) ---------------------------------------
 * Marks, for every string in bytes[str_off[0] .. str_off[n_str]), the first byte of each of
 * its chunks in the bitmap chunk_bits (bit i of word i/64, LSB first; offsets are relative
 * to str_off[0]).  chunk_bits must hold ceil(n_bytes/64) words.  Multithreaded over
 * strings (n_threads <= 0: all hardware threads, capped at 64).  Returns the chunk count
 * or a negative status. */
int64_t sw_presplit_host(const uint8_t* bytes, const int64_t* str_off, int64_t n_str, int32_t pattern,
                         uint64_t* chunk_bits, int32_t n_threads);

/* ---- special tokens (E1: special_tokens, shredword/base.py:103, saved/loaded at :120-121 /
 * :142-144; the reference defines no split) ----------------------------------------------------
 * The tokenizer's specials: their UTF-8 bytes[off[k] .. off[k+1]) and ids[k], in dict order.
 * Build-defined rule (minbpe's): scanning a string left to right, the first position where some
 * special matches starts an occurrence; at one position the first special in dict order wins;
 * the scan goes on after it.  An occurrence is one chunk that encodes to the special's id, and
 * the text between occurrences is encoded on its own (pre-split included).  Empty specials never
 * match.  Occurrences never cross a string. */
typedef struct sw_specials {
  const uint8_t* bytes;
  const int64_t* off;   /* [n + 1] */
  const int32_t* ids;   /* [n] */
  int64_t n;
} sw_specials;

/* The occurrences in the strings bytes[str_off[s] .. str_off[s+1]), found on host threads
 * (n_threads <= 0: all, capped at 64): sp_pos[k] (byte offset relative to str_off[0],
 * ascending), sp_len[k], sp_id[k].  cap == 0 only counts.  Returns the number of occurrences,
 * SW_ERR_CAP if more than cap, or another negative status. */
int64_t sw_find_specials_host(const uint8_t* bytes, const int64_t* str_off, int64_t n_str, const sw_specials* sp,
                              int64_t* sp_pos, int32_t* sp_len, int32_t* sp_id, int64_t cap, int32_t n_threads);

/* The same occurrences found on the device.  sw_encoder_set_specials uploads the specials to the
 * handle (once; calls with the same specials are free; NULL or n == 0 clears them).  Then
 * sw_find_specials_device scans d_bytes[d_str_off[s] .. d_str_off[s+1]) (device arrays, as
 * sw_encode_device takes them) and writes the occurrences to d_pos / d_len / d_id (positions
 * relative to d_bytes, ascending) and their number to d_count (device int64), asynchronously on
 * `stream`; n_host (optional) synchronises and receives the count.  cap >= n_bytes / (length of the
 * shortest non-empty special) is required (SW_ERR_CAP: that many occurrences fit at most).  Every
 * special must be <= 64 bytes (SW_ERR_ARG otherwise: the host finder takes any length).  The
 * outputs feed sw_encode_device_ex (sp_pos, sp_len, sp_id, n_sp = cap, d_n_sp = d_count) with no
 * synchronisation in between. */
int32_t sw_encoder_set_specials(sw_encoder* h, const sw_specials* sp);
int32_t sw_find_specials_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                                int64_t n_str, int64_t* d_pos, int32_t* d_len, int32_t* d_id, int64_t cap,
                                int64_t* d_count, void* stream, int64_t* n_host);

/* sw_presplit_host with special-token occurrences (as sw_find_specials_host gives them): the
 * text between occurrences is pre-split on its own and each occurrence is one chunk.  Returns the
 * chunk count or a negative status. */
int64_t sw_presplit_host_specials(const uint8_t* bytes, const int64_t* str_off, int64_t n_str, int32_t pattern,
                                  const int64_t* sp_pos, const int32_t* sp_len, int64_t n_sp, uint64_t* chunk_bits,
                                  int32_t n_threads);

/* ---- batched encode, host buffers (the Tokenizer.encode / encode_batch path) ------------
 * Encodes n_str strings (bytes[str_off[s] .. str_off[s+1])) and writes their ids
 * concatenated into out_ids, with out_off[0..n_str] the per-string offsets.
 * chunk_bits: optional pre-split bitmap as produced by sw_presplit_host; NULL => the
 * library pre-splits with `pattern` (on the device; on the host threads with
 * SW_OPT_HOST_PRESPLIT).  out_cap >= total input bytes always suffices.
 * stats: optional.  Synchronous. */
int32_t sw_encode_batch(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                        int32_t pattern, const uint64_t* chunk_bits, int32_t* out_ids, int64_t out_cap,
                        int64_t* out_off, sw_stats* stats);

/* apply_regex (shredword/base.py:38-58) on the device: the chunk-start bitmap of the strings
 * d_bytes[d_str_off[s] .. d_str_off[s+1]) (device pointers on the encoder's device;
 * d_str_off[0] == 0, d_str_off[n_str] == n_bytes) into d_chunk_bits[ceil(n_bytes/64)], the
 * layout of sw_presplit_host.  Bit-identical to sw_presplit_host.  stream: a hipStream_t on
 * that device; NULL is the null stream (torch's default stream).  If n_chunks_host is not
 * NULL the call synchronises and stores the number of chunks. */
int32_t sw_presplit_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                           int64_t n_str, int32_t pattern, uint64_t* d_chunk_bits, void* stream,
                           int64_t* n_chunks_host);

/* ---- batched encode, device-resident buffers (bench / multi-GPU driver) -----------------
 * All pointers are device pointers on the encoder's device: d_bytes[n_bytes],
 * d_str_off[n_str+1] (relative to d_bytes, d_str_off[0] == 0, d_str_off[n_str] == n_bytes),
 * d_chunk_bits[ceil(n_bytes/64)] or NULL (then the device pre-splits with the SW_OPT_PATTERN
 * pattern first: the full path), d_out_ids[n_bytes], d_out_off[n_str+1].  One launch takes
 * n_bytes <= 2^30 - 64 (SW_ERR_ARG otherwise); sw_encode_batch splits larger batches between
 * strings by itself.
 * stream: a hipStream_t on that device; NULL is the null stream (torch's default stream, as
 * in every HIP library API).
 * Asynchronous: the work is enqueued on the stream.  n_tokens_host (optional) forces a
 * synchronisation and receives the total id count. */

int32_t sw_encode_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                         int64_t n_str, const uint64_t* d_chunk_bits, int32_t* d_out_ids, int64_t* d_out_off,
                         void* stream, int64_t* n_tokens_host);

/* ---- the same with per-call choices ---------------------------------------------------------
 * sw_encode_device with (ex == NULL: exactly sw_encode_device):
 *   struct_size  sizeof(sw_encode_ex) of the caller's header: any other value is refused
 *                (SW_ERR_ARG), so a caller built against another layout fails loudly
 *   flags        SW_EX_PATTERN: `pattern` holds this call's pattern; clear (a zero-initialised
 *                struct): the handle's SW_OPT_PATTERN
 *   chunk_bits   as d_chunk_bits above (NULL: the device pre-splits with the pattern)
 *   out_bits     32 (or 0): d_out_ids is int32_t*; 16: uint16_t* -- the multi-GPU driver's 16-bit
 *                transport (SW_INFO_IDS16 tables only, and never together with special-token
 *                occurrences: SW_ERR_ARG otherwise)
 *   sp_pos / sp_len / sp_id / n_sp   special-token occurrences (device arrays; sp_pos relative to
 *                d_bytes, ascending, non-overlapping, each inside one string; n_sp == 0: none), as
 *                sw_find_specials_host finds them: each is one chunk encoding to its id, and the
 *                device pre-split treats its ends as string boundaries (a caller bitmap must already:
 *                sw_presplit_host_specials)
 *   pattern      with SW_EX_PATTERN: the device pre-split's pattern for this call (SW_PAT_*).  Per
 *                call, so that callers sharing one handle with different patterns do not race on the
 *                option.
 *   d_n_sp       NULL, or the occurrence count in device memory (sw_find_specials_device's d_count,
 *                not read back by the host): n_sp is then the arrays' capacity, and the encode reads
 *                the count on the device -- the find + encode sequence needs no synchronisation */
#define SW_EX_PATTERN 1u
typedef struct sw_encode_ex {
  int32_t struct_size;
  uint32_t flags;
  const uint64_t* chunk_bits;
  int32_t out_bits;
  const int64_t* sp_pos;
  const int32_t* sp_len;
  const int32_t* sp_id;
  int64_t n_sp;
  int32_t pattern;
  const int64_t* d_n_sp;
} sw_encode_ex;
int32_t sw_encode_device_ex(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                            int64_t n_str, const sw_encode_ex* ex, void* d_out_ids, int64_t* d_out_off, void* stream,
                            int64_t* n_tokens_host);

/* sw_encode_batch with special tokens (specials NULL or empty: exactly sw_encode_batch): the
 * occurrences are found on the device launch by launch (sw_find_specials_device; SW_OPT_DEVICE_SPECIALS)
 * or on the host threads (sw_find_specials_host: a special over 64 bytes, a caller's bitmap, or the
 * host pre-split) -- the same occurrences either way; the pre-split is the
 * device's, or the host threads' with SW_OPT_HOST_PRESPLIT (chunk_bits from the caller must come
 * from sw_presplit_host_specials on the same specials).  Host buffers; synchronous. */
int32_t sw_encode_batch_ex(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str, int32_t pattern,
                           const uint64_t* chunk_bits, const sw_specials* specials, int32_t* out_ids, int64_t out_cap,
                           int64_t* out_off, sw_stats* stats);

/* ---- decode (build_vocab, shredword/base.py:60-79, and the byte join of a decode) --------
 * A decoder holds a vocabulary: token t's bytes are vocab_bytes[vocab_off[t] .. vocab_off[t+1])
 * for every t < n_vocab with defined[t] != 0; the other ids are not tokens, and decoding one is
 * an error (the reference's vocab[idx] raises KeyError).  The UTF-8 decoding of the bytes
 * (errors="replace") is the caller's: it is per string. */
typedef struct sw_decoder sw_decoder;
int32_t sw_decoder_create(const uint8_t* vocab_bytes, const int64_t* vocab_off, const uint8_t* defined,
                          int64_t n_vocab, int32_t device, sw_decoder** out);
void sw_decoder_destroy(sw_decoder* d);

/* The ids ids[id_off[s] .. id_off[s+1]) of n_str strings -> their bytes, concatenated into
 * out[out_cap], with out_off[0..n_str] the per-string offsets.  Host buffers; synchronous.
 * SW_ERR_ARG if an id is not in the vocabulary, SW_ERR_CAP if out_cap is too small. */
int32_t sw_decode_batch(sw_decoder* d, const int32_t* ids, const int64_t* id_off, int64_t n_str, uint8_t* out,
                        int64_t out_cap, int64_t* out_off);

/* The same on device buffers (d_id_off[0] == 0, d_id_off[n_str] == n_ids) on a stream (NULL:
 * the null stream).  Asynchronous unless n_bytes_host is given: then the call synchronises,
 * stores the byte count and reports the errors above. */
int32_t sw_decode_device(sw_decoder* d, const int32_t* d_ids, int64_t n_ids, const int64_t* d_id_off, int64_t n_str,
                         uint8_t* d_out, int64_t out_cap, int64_t* d_out_off, void* stream, int64_t* n_bytes_host);

/* Device time of the whole sw_encode_device pipeline (every kernel from k_tile_strings to
 * k_string_offsets, back to back on one stream), measured with a HIP event pair on that stream.
 * sw_encoder_set_timing(h, 1) starts a new accumulation window (one event pair per launch, no
 * host synchronisation per call); sw_encoder_last_kernel_ms returns the average device time per
 * launch over that window (it synchronises on the last event), or -1. */
int32_t sw_encoder_set_timing(sw_encoder* h, int32_t on);
double sw_encoder_last_kernel_ms(const sw_encoder* h);
/* the same for the classification kernel alone (k_split_classify, or k_classify with a caller's
 * bitmap): the pipeline's dominant kernel, timed by HIP events on the launch stream */
double sw_encoder_last_classify_ms(const sw_encoder* h);

/* What the last sw_encode_device launch did (synchronises on it): out4[0] chunks, out4[1] chunks
 * that went to the merge loop (references to a merge result: not a single byte, not in the
 * whole-chunk table), out4[2] distinct ones actually merged (after the in-launch dedupe),
 * out4[3] tiles.  For reports; outside any timed region. */
int32_t sw_encoder_last_counts(sw_encoder* h, int64_t* out4);

/* Diagnostic builds only (compiled with -DSW_STAMPS): device cycles summed over workgroups,
 * per phase: 0 k_classify stage+enumerate, 1 classify lookups, 2 slot/queue writes, 3 string
 * offsets, 4 k_merge_bucket N<16 (per block), 5 k_merge_bucket N>=16, 6 k_merge_long,
 * 8..11 k_compact: slots + reference list, result gathers, chained scan, expansion + strings.
 * out32 holds 32 values.  reset != 0 zeroes the counters.  Regular builds return SW_ERR_ARG. */
int32_t sw_encoder_phase_cycles(sw_encoder* h, double* out32, int32_t reset);

/* ---- multi-GPU reassembly (no reference counterpart: the reference has
 * no multi-device path) ------------------------------------------------------------------------
 * The gathered, padded buffers of a doc-sharded encode over `world` ranks -> the batch's ids and
 * string offsets, contiguous, on the device.  Rank r's ids are d_recv[r*width .. r*width +
 * counts[r]) (id_bits 16: the low 16 bits of each id, an unsigned value widened here; 32: int32)
 * and its string offsets d_recv_off[r*width_s .. r*width_s + n_strs[r]) (relative to its own
 * ids).  d_counts / d_n_strs: int64[world] device arrays (the counts all-gather); a count above
 * its width is taken as the width (the caller checks its bounds: shard.check_bounds).  Writes
 * d_out_ids[0 .. sum counts) and d_out_off[0 .. sum n_strs] (rank r's offsets plus the ids of the
 * ranks before it; the last one is the total), so d_out_ids must hold world*width ids and
 * d_out_off world*width_s + 1 offsets.  Asynchronous on `stream` (NULL: the null stream). */
int32_t sw_reassemble_device(const void* d_recv, int32_t id_bits, const int64_t* d_counts, int64_t width,
                             const int64_t* d_recv_off, const int64_t* d_n_strs, int64_t width_s, int32_t world,
                             int32_t* d_out_ids, int64_t* d_out_off, void* stream);

/* ---- synthetic corpora (bench inputs; deterministic for any thread count) --------------
 * Fills out_off[0..n_strings] with string offsets; when out_bytes is non-NULL also writes
 * the bytes (cap >= out_off[n_strings]).  Returns the total byte count or SW_ERR_*. */
int64_t sw_synth_corpus(uint64_t seed, int32_t kind, int64_t n_strings, int64_t mean_len,
                        uint8_t* out_bytes, int64_t cap, int64_t* out_off, int32_t n_threads);

/* A corpus (bytes, off[0..n_strings]) with special tokens inserted: about per_kib random ones per
 * KiB of each string, each at a random code-point boundary, and sp's end_special-th one at every
 * string's end (end_special < 0: none).  Two passes like sw_synth_corpus (out_bytes NULL: only the
 * offsets).  Returns the total byte count or -1. */
int64_t sw_synth_splice_specials(uint64_t seed, const uint8_t* bytes, const int64_t* off, int64_t n_strings,
                                 const sw_specials* sp, double per_kib, int32_t end_special, uint8_t* out_bytes,
                                 int64_t cap, int64_t* out_off, int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif
