/* shredword_train.h -- C-ABI of the MI355X-accelerated BPE trainer.
 *
 * The trainer the reference ships as its C++ core (shredword/csrc/bpe/, C API bpe.h:62-72,
 * bound by ctypes in shredword/cbase.py:44-59 and wrapped by shredword/trainer.py), with the
 * two corpus-wide passes on the GPU:
 *   - the pair histogram (bpe_count_bigrams, bpe.cpp:315-370): one device hash table of pair
 *     frequencies and first occurrences, filled by every word at once;
 *   - the per-merge rewrite (bpe_merge_batch, bpe.cpp:437-483): every word rewritten in place
 *     on the device, the neighbour-pair frequency changes accumulated in a device hash table.
 * The host keeps what is sequential by nature (the max-heap with lazy versions, bpe.cpp:405-
 * 529, heap.cpp) and applies each merge's changes in the reference's own order, so the merges
 * are the reference's, bit for bit (oracle/sw_train_oracle.c restates them; tests/golden/
 * train_* pin both to the reference trainer's output).  Two reference defects are fixed: no
 * symbol starts "deleted" (histogram.cpp:14-22 leaves the flag uninitialised) and token
 * frequencies skip a negative unk_id (bpe.cpp:709 writes freq[-1]).
 *
 * Status codes and sw_last_error() as in shredword_hip.h (the same library).
 */
#ifndef SHREDWORD_TRAIN_H
#define SHREDWORD_TRAIN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Field for field the reference's BPEConfig (bpe.h:43-48; ctypes mirror cbase.py:40), so a
 * binding written for create_trainer() passes the same structure.  character_coverage outside
 * (0, 1) means 0.995 and min_pair_freq 0 means 2000, as create_trainer does (bpe.cpp:124-130). */
typedef struct sw_train_config {
  size_t target_vocab_size;
  int32_t unk_id;
  float character_coverage;
  uint64_t min_pair_freq;
} sw_train_config;

typedef struct sw_trainer sw_trainer;

/* create_trainer (bpe.cpp:112-136) on HIP device `device`.  SW_ERR_NODEV without a GPU. */
int32_t sw_trainer_create(const sw_train_config* config, int32_t device, sw_trainer** out);
/* bpe_trainer_destroy (bpe.cpp:148-158).  NULL is a no-op. */
void sw_trainer_destroy(sw_trainer* t);

/* bpe_load_corpus (bpe.cpp:208-297): words are the maximal runs of bytes other than ' ', '\t',
 * '\r', '\n'; the corpus is their distinct set with counts, characters outside the coverage
 * mapped to unk_id.  From a file, or from memory.  Text with NUL bytes is refused (SW_ERR_ARG). */
int32_t sw_trainer_load_corpus(sw_trainer* t, const char* path);
int32_t sw_trainer_load_text(sw_trainer* t, const uint8_t* text, int64_t n);

/* bpe_train (bpe.cpp:597-655): merges until target_vocab_size - 256 of them or no pair is left
 * at min_pair_freq.  Returns the number of merges performed (>= 0) or a negative status. */
int64_t sw_trainer_train(sw_trainer* t);

/* The merges as (left id, right id, new id) int32 rows, new id = 256 + row (bpe.cpp:424);
 * returns their number (rows beyond cap are not written). */
int64_t sw_trainer_merges(const sw_trainer* t, int32_t* rows, int64_t cap);
/* Final token frequencies [256 + merges] over the rewritten corpus (bpe_save, bpe.cpp:703-712);
 * returns their number. */
int64_t sw_trainer_token_freq(const sw_trainer* t, uint64_t* freq, int64_t cap);

/* bpe_save (bpe.cpp:678-739): model_path gets the merges as raw int32 triples, vocab_path one
 * "token frequency" line per id with the token as a C string (as the reference writes them).
 * Either path may be NULL. */
int32_t sw_trainer_save(const sw_trainer* t, const char* model_path, const char* vocab_path);

/* Timing of the last load + train (ms): [0] corpus load (host), [1] upload, [2] pair histogram
 * (device) + heap seed, [3] host time spent waiting for the merge rewrites on the device (sum),
 * [4] host work on the critical path: pops, launches, change application not hidden behind a
 * merge launched ahead (sum), [5] merges, [6] distinct words, [7] symbols. */
int32_t sw_trainer_stats(const sw_trainer* t, double* out8);

#ifdef __cplusplus
}
#endif
#endif
