/*
 * gpubpe.h — C-ABI of the MI355X-native BPE train + trie-encode engine.
 *
 * This is the drop-in boundary for the reference's WebGPU device layer
 * (toprakdeviren/gpu-bpe: src/bpe/engine.js + the WGSL kernels in
 * src/bpe/train.wgsl and src/bpe/tokenizer/tokenize.wgsl).  A host binding
 * (the Node N-API addon in gpu-bpe_amd/js/, the Python ctypes binding in
 * gpu-bpe_amd/gpubpe/) wraps these entry points and keeps the reference's
 * JavaScript API (BPEEngine / BPETrainer / TrieTokenizer).
 *
 * Conventions
 *  - Plain C types only; no HIP or torch types cross the boundary.
 *  - Every function returns an int status (GBPE_OK = 0, negatives = errors);
 *    gbpe_last_error(ctx) returns a message for the last failure on ctx.
 *  - The caller owns every host buffer; buffers are borrowed for the call
 *    and never retained.  The library owns and pools device memory.
 *  - A context is bound to one HIP device and one stream; it is not
 *    re-entrant (one thread at a time), like the reference's single queue.
 *  - Symbols in and out use the reference layout: u32, bits[15:0] = token
 *    id, bit 16 = word start (train.wgsl:36-37).
 */
#ifndef GPUBPE_H
#define GPUBPE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GBPE_ABI_VERSION 5   /* 5: paired_merges added to the stats, gbpe_ctx_trim (round 6); 4: the late-loop
                                 stats removed, trainer creation time added (round 5) */

/* status codes */
#define GBPE_OK            0
#define GBPE_E_INVALID    -1   /* bad argument */
#define GBPE_E_OOM        -2   /* device or host allocation failed */
#define GBPE_E_DEVICE     -3   /* HIP runtime / kernel failure */
#define GBPE_E_CAPACITY   -4   /* output buffer too small; required size returned */
#define GBPE_E_CANCELLED  -5   /* progress callback returned non-zero */
#define GBPE_E_EMPTY      -6   /* empty corpus (trainer.js:161-163) */
#define GBPE_E_INTERNAL   -7   /* invariant violated (reported, never silent) */

/* reference constants (engine.js:10-13, training-pipeline.js:13) */
#define GBPE_WORKGROUP_SIZE   256u
#define GBPE_TABLE_SIZE       2097152u
#define GBPE_INVALID_TOKEN    0xFFFFFFFFu
#define GBPE_BATCH_SIZE       128u
#define GBPE_WORD_START_BIT   0x10000u

typedef struct gbpe_ctx gbpe_ctx;
typedef struct gbpe_trainer gbpe_trainer;
typedef struct gbpe_trie gbpe_trie;

/* ── context / device (replaces engine.js:143-177 requestGPUDevice and
 *    engine.js:216-238 BPEEngine.init) ─────────────────────────────────── */
int  gbpe_ctx_create(int device_ordinal, gbpe_ctx** out);
void gbpe_ctx_destroy(gbpe_ctx* ctx);
/* Give the context's idle pooled device / pinned blocks back to the runtime (the
   pool keeps freed trainer buffers for the next trainer, tokenizer.js:30-46): for
   callers about to allocate outside the library (no reference counterpart). */
int gbpe_ctx_trim(gbpe_ctx* ctx);
/* engine.js:207-210 `limits.maxBufferSize` (used by tokenizer.js:181 for
 * multi-pass slicing).  This engine has no per-buffer cap below HBM size. */
int  gbpe_ctx_limits(gbpe_ctx* ctx, uint64_t* max_buffer_size);
const char* gbpe_last_error(const gbpe_ctx* ctx);
const char* gbpe_version(void);
/* GBPE_ABI_VERSION the library was built with, and sizeof(gbpe_trainer_stats) there:
 * a caller built against another header checks both before gbpe_trainer_stats_get */
int gbpe_abi_version(void);
uint64_t gbpe_trainer_stats_size(void);
/* number of compiled kernels (engine.js:234 logs Object.keys(pipelines).length) */
int  gbpe_kernel_count(void);
const char* gbpe_kernel_name(int i);

/* ── word boundaries (train.wgsl:144-186 bpe_word_boundary) ──────────────
 * ws_out[i] = 1 if byte i starts a word under the reference byte-class
 * heuristic. */
int gbpe_word_boundary(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, uint8_t* ws_out);

/* PreTokenizer.preTokenizeBytes (src/wasm/pre_tokenizer.mjs:459-509) word-start
 * mask for NFC UTF-8 bytes (the reference also NFC-normalises: identity on NFC
 * input).  Classes: Unicode general categories (unicode_classes.h). */
int gbpe_pretokenize_gpt4(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, uint8_t* ws_out);
int gbpe_pretokenize_gpt4_device(gbpe_ctx* ctx, const void* d_bytes, uint64_t n, void* d_ws);

/* ── training (replaces trainer.js:149-335 BPETrainer.train over the
 *    train.wgsl kernels, training-pipeline.js:178-222 encodeBatch) ─────── */

/* Reproduce the reference's compaction exactly (default, 0) or use the
 * intended compaction.  The reference bounds bpe_finalize_compact_b with
 * the already-updated symbol count (train.wgsl:605-607, 698, 727) so the
 * last m slots of each compacted stream keep stale ping-pong contents. */
#define GBPE_TRAIN_EXACT_COMPACTION  (1u << 0)
/* record per-kernel device time with HIP events (read via gbpe_trainer_stats) */
#define GBPE_TRAIN_TIMING            (1u << 1)
/* word starts from the GPT-4 rules of the reference's PreTokenizer
 * (src/wasm/pre_tokenizer.mjs:226-292) computed on the device, for NFC UTF-8
 * input; ignored when word_starts is given */
#define GBPE_TRAIN_GPT4_BOUNDARIES   (1u << 2)
/* Sector-sparse merge loop.  Once the merge counts have fallen
 * far below the stream length, the stream is re-laid out as word-aligned
 * sectors with a token-presence bitmap: a merge then touches only the sectors
 * holding both of its tokens, plus a dense zone at the end of the stream that
 * carries the reference's compaction quirk.  On by default (same results as
 * the dense loop); DENSE_ONLY disables it, SPARSE_EARLY enters it at the first
 * step boundary where the zone fits (tests). */
#define GBPE_TRAIN_DENSE_ONLY        (1u << 3)
#define GBPE_TRAIN_SPARSE_EARLY      (1u << 4)

typedef struct gbpe_train_opts {
    uint32_t target_vocab_size;  /* trainer.js:149 targetVocabSize (reference default 4096) */
    uint32_t vocab_size;         /* Vocab.size before training (256 for a fresh Vocab) */
    uint32_t next_token_id;      /* Vocab.nextTokenId (trainer.js:191) */
    uint32_t batch_size;         /* merges per host round trip; 0 = 128 (training-pipeline.js:13) */
    uint32_t flags;              /* GBPE_TRAIN_* */
    uint32_t table_log2;         /* pair-table slots = 2^table_log2; 0 = automatic */
} gbpe_train_opts;

typedef struct gbpe_progress {   /* trainer.js:306-315 onProgress payload */
    uint32_t merge_index;        /* totalMergesDone */
    uint32_t total_merges;       /* mergesNeeded */
    uint32_t best_count;         /* count of the batch's last merge */
    uint32_t symbol_count;       /* current stream length */
    uint32_t batch_merges;       /* merges in this batch */
    uint32_t early_stop;
    double   elapsed_s;          /* since the loop started (trainer.js:230, 291) */
} gbpe_progress;

/* Called once per batch with that batch's merges as [a, b, id, count] x
 * batch_merges.  Return non-zero to cancel (gbpe_train returns
 * GBPE_E_CANCELLED, merges so far are kept). */
typedef int (*gbpe_progress_cb)(const gbpe_progress* p, const uint32_t* batch, void* user);

/* One-shot training from host bytes.  word_starts may be NULL (use the
 * heuristic kernel, trainer.js:177-180) or a byte mask (trainer.js:115-121).
 * merges_out receives [a, b, id, count] x n_merges (capacity merges_cap).
 * Returns GBPE_E_EMPTY for n == 0. */
int gbpe_train(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
               const gbpe_train_opts* opts, gbpe_progress_cb cb, void* user,
               uint32_t* merges_out, uint32_t merges_cap, uint32_t* n_merges, uint32_t* early_stop);

/* Stepwise trainer.  With input_on_device != 0, `bytes` (and `word_starts`)
 * are device pointers already resident in HBM (bench path). */
int gbpe_trainer_create(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                        int input_on_device, const gbpe_train_opts* opts, gbpe_trainer** out);
/* Run up to max_merges merges (one host sync).  merges_out may be NULL. */
int gbpe_trainer_step(gbpe_trainer* t, uint32_t max_merges, uint32_t* merges_out,
                      uint32_t* n_done, uint32_t* early_stop);

typedef struct gbpe_trainer_stats {
    uint64_t symbol_count;        /* current stream length */
    uint64_t merges_done;         /* total merges so far */
    uint64_t stream_bytes_moved;  /* sum over merges of s*(2*N_i + N_{i+1}), s = bytes/symbol */
    uint64_t tail_dropped;        /* sum of m over merges (reference compaction quirk) */
    uint64_t live_pairs;          /* distinct pairs with count > 0 (last refresh) */
    uint64_t table_slots;
    uint64_t table_used;          /* occupied slots (incl. dead) */
    uint64_t max_live_pairs;      /* max over merges: > ~1.7M means the reference's 2^21
                                     table would likely have dropped counts (train.wgsl:422-429) */
    uint32_t bytes_per_symbol;
    uint32_t early_stop;
    double   ms_merge;            /* GBPE_TRAIN_TIMING: device ms in the two stream kernels (k_delta + k_compact) */
    double   ms_select;           /* k_select: argmax + merge setup */
    double   ms_other;            /* k_refresh: block maxima of touched table blocks */
    uint64_t timed_merges;
    double   ms_delta;            /* k_delta alone (HIP events between the two stream kernels) */
    double   ms_compact;          /* k_compact alone (tiles + stale-tail blocks) */
    uint64_t sparse_merges;       /* merges run by the sector-sparse loop */
    uint32_t sparse_enters;       /* dense -> sparse re-layouts */
    uint32_t sparse_exits;        /* sparse -> dense re-layouts (export, zone too small; a crowded table grows in place) */
    uint64_t sparse_sectors;      /* sectors of the last sparse layout */
    uint64_t sparse_zone;         /* zone length at the last sparse entry */
    uint64_t body_bytes;          /* bytes k_body actually moved: candidate extents + signature words, sector
                                     symbols read and rewritten, the single-workgroup zone pass (pair-table
                                     traffic excluded) */
    uint64_t zone_bytes;          /* bytes of the multi-tile zone passes (zone k_delta + k_compact + window copy) */
    uint64_t dense_bytes;         /* s*(2*N_i + N_{i+1}) summed over the dense merges only */
    double   ms_dense;            /* GBPE_TRAIN_TIMING: merge-pass device ms of the dense merges (k_delta + k_compact) */
    double   ms_sparse;           /* GBPE_TRAIN_TIMING: merge-pass device ms of the sparse merges (k_body + zone passes) */
    double   ms_body;             /* GBPE_TRAIN_TIMING: k_body alone */
    uint32_t lexicon_builds;      /* sparse entries whose body became a word lexicon */
    uint32_t lexicon_fallbacks;   /* ... that kept the in-place sectors (store not much smaller, collision) */
    uint64_t lexicon_words;       /* body word occurrences the lexicon represents (all builds and shrinks) */
    uint64_t lexicon_entries;     /* distinct-word entries of the current lexicon */
    uint64_t lexicon_symbols;     /* symbols of the current lexicon store (separators included) */
    double   ms_create;           /* host wall ms of trainer creation (symbols, word starts, first count):
                                     the part of a run the reference's t_loop excludes (trainer.js:230) */
    uint64_t paired_merges;       /* merges run as the second merge of a paired k_body launch */
} gbpe_trainer_stats;
int gbpe_trainer_stats_get(gbpe_trainer* t, gbpe_trainer_stats* out);
/* Current symbol stream in the reference u32 layout (bit16 = word start). */
int gbpe_trainer_symbols(gbpe_trainer* t, uint32_t* out, uint64_t cap, uint64_t* n);
/* Live pair counts (count > 0): pids[i] = a<<16|b.  For parity tests. */
int gbpe_trainer_pair_counts(gbpe_trainer* t, uint32_t* pids, uint32_t* counts, uint64_t cap, uint64_t* n);
void gbpe_trainer_destroy(gbpe_trainer* t);

/* The library's HIP stream (the lexicon hand-over runs RCCL transfers on it). */
int gbpe_ctx_set_stream(gbpe_ctx* ctx, void* hip_stream);   /* taken literally (NULL = the null stream) */
void* gbpe_ctx_get_stream(gbpe_ctx* ctx);                    /* current stream (save / restore) */
/* ── checkpoint / resume: a run continues on another trainer ─────────────────
 * (The reference keeps no mid-run checkpoint)  The
 * state of a trainer is its current stream and its previous stream (the
 * ping-pong buffer the compaction quirk reads stale symbols from,
 * train.wgsl:605-607 + 698/727), both in the reference u32 layout (bit16 =
 * word start).  cur/prev NULL = lengths only; on_device != 0: cur/prev are
 * device pointers.
 * `prev` is defined only where the next merge's stale window can read it: after
 * the sector-sparse loop, positions below the body length at its last merge hold
 * the body as it was at entry, not the previous stream (the window always lies in
 * the stream's tail, so a resumed run reads the same symbols). */
int gbpe_trainer_export_state(gbpe_trainer* t, uint32_t* cur, uint64_t cap_cur, uint64_t* n_cur,
                              uint32_t* prev, uint64_t cap_prev, uint64_t* n_prev, int on_device);
/* A single-device trainer continuing from an exported state: opts as for
 * gbpe_trainer_create with vocab_size / next_token_id of the run so far (the
 * merges still to do are target_vocab_size - vocab_size); pair counts are
 * recounted from `cur`.  n_prev >= n (n_prev - n is the last merge's count;
 * n_prev == n for a run with no merges yet, whose prev is all zero). */
int gbpe_trainer_create_from_state(gbpe_ctx* ctx, const uint32_t* cur, uint64_t n, const uint32_t* prev,
                                   uint64_t n_prev, int input_on_device, const gbpe_train_opts* opts,
                                   gbpe_trainer** out);

/* ── sharded first pass + lexicon hand-over ─────────
 * The reference trains on one device (training-pipeline.js:178-222) and its merge
 * chain is sequential, so a multi-GPU run parallelises the first pass instead:
 * every rank turns ITS piece of the corpus (cut at a word start of the global
 * stream, the pieces concatenated in rank order are the corpus) into symbols, pair
 * counts and a word lexicon — its distinct words with their multiplicities — and ONE
 * root continues from all of them with the single-device sector-sparse loop
 * (DESIGN §2b/§2c).  The stream's tail — the last zt symbols, cut at a word start;
 * it may span several pieces — stays dense as the zone, where the reference
 * compaction quirk acts (train.wgsl:605-607 + 698/727).  The stream order
 * of the body stays on the ranks (their occurrence lists), so the stream may exceed
 * one device's 32-bit positions (C4: 8.6*10^9 symbols).  Protocol:
 *   rank:  lexshard_create → info_get: top_count, symbols → (sum of top counts: an upper
 *          bound of the first merge's count → zt; this piece's part of the last zt
 *          stream symbols) lexshard_build(part) → copy STORE + MUL + ZONE to the root
 *          → release
 *   root:  trainer_create_from_lexicon(stores in rank order, zones in rank order,
 *          body symbols)
 *          → map (a global word id per store entry, in rank order) → rank slices
 *          → lexshard_remap; gbpe_trainer_step as for any trainer
 *   check: gbpe_trainer_expand(root, every rank's OCC in rank order) = the stream. */
typedef struct gbpe_lexshard gbpe_lexshard;
typedef struct gbpe_lexshard_info {
    uint64_t symbols;        /* the piece's symbols */
    uint64_t body;           /* symbols before its zone (all of them on a rank without a zone) */
    uint64_t zone;           /* zone symbols (the ranks holding the stream's tail) */
    uint64_t store_symbols;  /* distinct words + one 0 separator each */
    uint64_t entries;        /* distinct words (words over 64 symbols: one entry per occurrence) */
    uint64_t words;          /* body words in stream order (the occurrence list) */
    uint32_t top_count;      /* the piece's largest pair count */
    uint32_t bytes_per_symbol;   /* STORE / ZONE layout: 2 = u16 (bit 15 word start), 4 = u32 (bit 16) */
} gbpe_lexshard_info;
#define GBPE_LEXSHARD_STORE 0   /* store_symbols x bytes_per_symbol */
#define GBPE_LEXSHARD_MUL   1   /* store_symbols x u32: each symbol's word multiplicity (0 at separators) */
#define GBPE_LEXSHARD_OCC   2   /* words x u32: word id (local; global after remap) or 0x80000000|symbol */
#define GBPE_LEXSHARD_ZONE  3   /* zone x bytes_per_symbol */
/* opts as for gbpe_trainer_create, identical on every rank and the root */
int  gbpe_lexshard_create(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                          int input_on_device, const gbpe_train_opts* opts, gbpe_lexshard** out);
int  gbpe_lexshard_build(gbpe_lexshard* ls, uint64_t zone_target /* 0: no zone; >= symbols: all zone */);
int  gbpe_lexshard_info_get(const gbpe_lexshard* ls, gbpe_lexshard_info* out);
int  gbpe_lexshard_copy(gbpe_lexshard* ls, int part, void* dst, uint64_t cap_bytes, int dst_on_device);
int  gbpe_lexshard_release(gbpe_lexshard* ls);   /* frees the piece's stream and counts, keeps the lexicon */
int  gbpe_lexshard_remap(gbpe_lexshard* ls, const uint32_t* map, uint64_t n_map, int map_on_device);
void gbpe_lexshard_destroy(gbpe_lexshard* ls);
/* The root trainer: store / mul = every rank's STORE and MUL concatenated in rank
 * order (store_len symbols), zone = every rank's ZONE in rank order, body_len = the symbols of
 * every piece before the zone (the stream is body_len + zone_len symbols; may exceed
 * 2^32).  map_out (map_cap entries) receives one global word id per store entry.
 * The trainer never returns to one dense stream: gbpe_trainer_symbols /
 * export_state fail, gbpe_trainer_expand rebuilds the stream. */
int  gbpe_trainer_create_from_lexicon(gbpe_ctx* ctx, const void* store, const uint32_t* mul, uint64_t store_len,
                                      const void* zone, uint64_t zone_len, uint64_t body_len, int input_on_device,
                                      const gbpe_train_opts* opts, uint32_t* map_out, uint64_t map_cap,
                                      uint64_t* n_map, int map_on_device, gbpe_trainer** out);
/* The current stream (u32 reference layout) of a trainer in the word-lexicon loop:
 * prefix_occ (every rank's remapped OCC in rank order; none for a single-device
 * trainer) then the trainer's own occurrences, then its zone.  out NULL: length only. */
int  gbpe_trainer_expand(gbpe_trainer* t, const uint32_t* prefix_occ, uint64_t n_prefix, int prefix_on_device,
                         uint32_t* out, uint64_t cap, uint64_t* n_out, int out_on_device);

/* ── trie encode (replaces tokenizer.js:54-335 TrieTokenizer over the
 *    tokenize.wgsl kernels) ─────────────────────────────────────────────── */

/* Upload a parsed trie (trie.js:137-160 parseTrieBuffers output): nodes =
 * u32 x 3 per node {firstChild, numChildren, tokenId}, edges = u32 x 2 per
 * edge {symbol, targetNode}.  Replaces tokenizer.js:59-71. */
/* native compileVocabToTrie (trie.js:39-98 + serializeTrie :167-206): token id i
 * has bytes[offsets[i] .. offsets[i+1]) (empty = skipped); writes the v3 blob.
 * out == NULL: *out_len = the size needed.  Host only (no context). */
int  gbpe_trie_compile(const uint8_t* bytes, const uint64_t* offsets, uint32_t n_tokens, uint8_t* out, uint64_t cap,
                       uint64_t* out_len);
/* DXFT .bin (export-controller.js:221-248): u32 [0x44584654, vocabSize,
 * tokenCount, vocabJsonLen] + tokens + vocab JSON bytes.  out == NULL: size only. */
int  gbpe_dxft_pack(const uint32_t* tokens, uint64_t n_tokens, uint32_t vocab_size, const uint8_t* vocab_json,
                    uint64_t json_len, uint8_t* out, uint64_t cap, uint64_t* out_len);
int  gbpe_trie_upload(gbpe_ctx* ctx, const uint32_t* nodes, uint32_t n_nodes,
                      const uint32_t* edges, uint32_t n_edges, gbpe_trie** out);
void gbpe_trie_free(gbpe_trie* trie);
/* double-array size of the uploaded trie; maxTokenLen (tokenizer.js maxTokenLen getter) and max id */
int  gbpe_trie_info(const gbpe_trie* trie, uint32_t* n_records, uint32_t* max_token_len, uint32_t* max_token_id);

/* tokenizer.js:173-206 encodeBytes: chunked greedy longest match.
 * chunk_size 0 = the reference's adaptive size (tokenizer.js:67-68).
 * On GBPE_E_CAPACITY *n_out holds the required token count. */
int gbpe_encode(gbpe_ctx* ctx, gbpe_trie* trie, const uint8_t* bytes, uint64_t n, uint32_t chunk_size,
                uint32_t* out, uint64_t out_cap, uint64_t* n_out);
/* Device-resident variant: d_bytes / d_out are device pointers (bench path). */
int gbpe_encode_device(gbpe_ctx* ctx, gbpe_trie* trie, const void* d_bytes, uint64_t n, uint32_t chunk_size,
                       void* d_out, uint64_t out_cap, uint64_t* n_out);
/* device ms of the last encode's kernels (walk, scan, compact) */
/* ── merge-rank encode: TokenizerManager.encode (tokenizer-manager.js:13-61) ──
 * merges = [a, b, newId] x n in learned order.  Exact for any merge list: a
 * merge whose operand is only created later never fires (as in the reference). */
typedef struct gbpe_bpe gbpe_bpe;
int  gbpe_bpe_upload(gbpe_ctx* ctx, const uint32_t* merges, uint32_t n_merges, gbpe_bpe** out);
int  gbpe_bpe_encode(gbpe_ctx* ctx, gbpe_bpe* bpe, const uint8_t* bytes, uint64_t n, uint32_t* out, uint64_t out_cap,
                     uint64_t* n_out);
void gbpe_bpe_free(gbpe_bpe* bpe);

int gbpe_encode_last_timing(gbpe_ctx* ctx, double* ms_walk, double* ms_scan, double* ms_compact);

/* ── device memory helpers for device-resident callers ─────────────────── */
int gbpe_device_alloc(gbpe_ctx* ctx, uint64_t bytes, void** dptr);
int gbpe_device_free(gbpe_ctx* ctx, void* dptr);
int gbpe_memcpy_h2d(gbpe_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int gbpe_memcpy_d2h(gbpe_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int gbpe_synchronize(gbpe_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* GPUBPE_H */
