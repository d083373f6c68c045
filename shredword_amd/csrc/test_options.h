// The library's measurement and test switches (sw_encoder_set_option): ablations and limits the
// benchmark and the tests set.  Not part of the public interface (include/shredword_hip.h lists
// the user-facing options); every one of them leaves the results unchanged.
#pragma once

// SW_OPT_CHUNK_TABLE  1 (default): a chunk of 2..16 bytes that encodes to exactly one token is
//                     answered from the whole-chunk table; 0: every chunk runs the merge loop
// SW_OPT_DEDUPE       1 (default): within one launch, a chunk whose bytes already occurred shares the
//                     first occurrence's merge result (bytes compared); 0: every occurrence merges
#define SW_OPT_CHUNK_TABLE 1
#define SW_OPT_DEDUPE 2
// SW_OPT_DEDUPE_SLOTS    cap on the dedupe table's slots (0 = automatic, else a power of two >= 8)
// SW_OPT_DEDUPE_FP_BITS  fingerprint bits compared before the bytes (26 = default; 0: every probe
//                        falls through to the byte comparison)
// SW_OPT_DEDUPE_EXACT    1 (default): keys of chunks up to 7 bytes are the bytes themselves; 0: every
//                        key is a verified fingerprint
#define SW_OPT_DEDUPE_SLOTS 3
#define SW_OPT_DEDUPE_FP_BITS 4
#define SW_OPT_DEDUPE_EXACT 10
// SW_OPT_LONG_SPLIT      1 (default): long chunks of well-formed tables take split + verify (long_split.h);
//                        0: one wave loop per chunk
#define SW_OPT_LONG_SPLIT 7
// SW_OPT_PIPE_COPY_KERNELS  1 (default): the pipeline's PCIe copies are kernels; 0: DMA copies
#define SW_OPT_PIPE_COPY_KERNELS 11
// SW_OPT_MERGE_STREAMS   1 (default): the merge buckets run on forked streams; 0: in order
#define SW_OPT_MERGE_STREAMS 13
// SW_OPT_FUSED_PRESPLIT  1 (default): the device pre-split inside the classification; 0: its own kernel
#define SW_OPT_FUSED_PRESPLIT 14
// SW_OPT_TEST_FAIL_GROWTH  1: the dedupe table's next growth allocation fails (the encoder must keep the
//                          table it has)
#define SW_OPT_TEST_FAIL_GROWTH 17
// SW_OPT_COMPACT_KERNEL  the id compaction kernel: 0 (default) picks from the previous launch's ids per
//                        tile; 1: 6 waves per SIMD, 1024 ids staged; 2: 7 waves, 768 staged; 3: as 2 with
//                        typed LDS / global accesses
#define SW_OPT_COMPACT_KERNEL 19
// SW_OPT_STAGED_HEADS    0 (default): k_tile_count stages the result heads for k_compact when the dedupe table
//                        has grown (low-repetition text); 1: always; 2: never
#define SW_OPT_STAGED_HEADS 20
