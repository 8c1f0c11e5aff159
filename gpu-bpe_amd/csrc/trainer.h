// Host side of the trainer shared by the training translation units: the
// gbpe_trainer object and the helpers that lay out and re-lay out its state
// (pair table, sector-sparse layout, word lexicon, zone).  See train.hip.
#pragma once

#include <cmath>

#include "train_dev.h"
#include <chrono>
#include "sparse.h"


// ─── host side ──────────────────────────────────────────────────────────────


struct gbpe_trainer {
    gbpe_ctx* ctx = nullptr;
    bool u16 = true;
    uint32_t bps = 2;            // bytes per symbol
    uint64_t n0 = 0, cap_syms = 0;
    uint64_t n_prev0 = 0;        // created from a state: its previous-stream length (export before any merge)
    uint32_t next_id0 = 256;     // Vocab.nextTokenId at creation
    void* buf[2] = {nullptr, nullptr};
    int cur = 0;                 // index of the buffer holding the stream
    uint64_t n = 0;              // host copy of the stream length (the device state holds it modulo 2^32:
                                 // a lexicon trainer built from shards may exceed 32 bits)
    uint32_t needed = 0, done = 0;
    bool stop = false;
    uint32_t flags = 0, batch = GBPE_BATCH_SIZE;
    DevState* st = nullptr;
    DevState* h_st = nullptr;    // pinned
    uint32_t* d_log = nullptr;
    uint32_t* h_log = nullptr;   // pinned
    Table tb{};
    uint32_t table_log2 = 22;
    uint32_t* hitmask = nullptr;
    uint32_t* tile_cnt = nullptr;
    uint32_t* grpsum = nullptr;
    // stats
    uint64_t bytes_moved = 0;
    uint64_t max_live = 0;
    double ms_merge = 0, ms_select = 0, ms_other = 0, ms_delta = 0, ms_compact = 0;
    uint64_t timed_merges = 0;
    std::vector<hipEvent_t> evs;
    // sector-sparse loop
    bool sp = false;             // the stream is in the sector layout
    uint32_t sp_secw = 256;      // sector window (symbols)
    uint32_t max_id = 0;         // exclusive bound of every token id of the run (bitmap rows)
    uint32_t last_mc = 0;        // count of the last merge run
    int bcur = 0;                // dense buffer holding the body sectors
    uint32_t nsec = 0;
    uint64_t nsec_cap = 0, loc_cap = 0;
    uint32_t bend = 0;           // end of the body's sector windows in the body buffer
    uint32_t sp_shrinks = 0;     // zone shrinks since the last entry
    uint2* sec = nullptr;        // {start, count} per sector
    uint32_t* sp_loc = nullptr;  // per-sector scratch (starts / scan)
    uint64_t* sp_blk = nullptr;  // scan block totals
    uint32_t* bits = nullptr;    // presence bitmap, rows = token ids, W words per row
    uint32_t* sig = nullptr;     // per-sector pair signatures (SP_SIGW words each)
    uint64_t sig_cap = 0;
    uint64_t sp_age = 0;         // sparse merges since the signatures were built
    uint64_t sp_bits_age = 0;    // ... since the token bitmap was built
    uint64_t bits_cap = 0;       // words
    uint32_t W = 0;
    void* zbuf[2] = {nullptr, nullptr};
    void* wtmp = nullptr;        // stale-window source copy
    uint64_t zcap = 0;           // zone buffer capacity (symbols)
    int zcur = 0;                // zone buffer holding the zone
    DevState* zst = nullptr;     // the zone's loop state
    DevState* h_zst = nullptr;   // pinned
    uint32_t* d_u32 = nullptr;   // small device scratch
    uint64_t* part = nullptr;    // k_refresh workgroup maxima (sparse selection)
    uint32_t grow_used_pct = 50;   // the table is rebuilt once its occupied slots (dead included) pass this %
    uint32_t grow_live_pct = 25;   // ... into the smallest 2^k slots its live pairs fill to at most this %
    uint2* zdr_out = nullptr;    // the multi-tile zone passes' delta dumps (ZdrView, train_dev.h)
    uint32_t* zdr_offs = nullptr;
    uint32_t* zdr_flag = nullptr;
    uint32_t zdr_ntile = 0;      // tile-workgroup dumps the buffers hold (+ ZDR_P churn workgroups)
    bool zdr_on = true;          // two-stage zone delta reduction (false: every workgroup flushes, the round-2 path)
    uint32_t* zseg = nullptr;    // ZSegState: the zone segments' per-merge hand-off (k_refresh zeroes it)
    uint32_t zseg_mode = 1;      // 1 = zone segments for zones beyond zone_one (up to 1M), 0 = off
    uint32_t table_grows = 0;    // crowded-table rebuilds (same size or larger)
    uint64_t* wg_bytes = nullptr;   // bytes moved per k_body workgroup (each its own counter)
    uint32_t delta_mt = 2048;       // dense k_delta: multi-tile workgroups from this many tiles (0 = never; GBPE_DEBUG delta_mt)
    uint32_t delta_tpw = 8;         // ... of 8, 16 or 32 tiles
    uint64_t wg_cap = 0;
    double ms_sparse = 0, ms_dense = 0;   // GBPE_TRAIN_TIMING: merge passes (without selection / refresh) by mode
    double ms_body = 0;          // GBPE_TRAIN_TIMING: k_body alone
    double ms_create = 0;        // host wall time of trainer creation
    uint64_t dense_bytes = 0;    // algorithmic stream bytes of the dense merges
    uint32_t g_refresh = 0;
    uint64_t sp_merges = 0, sp_sectors = 0, sp_zone = 0;
    uint32_t sp_enters = 0, sp_exits = 0;
    uint32_t sp_div = 64;        // enter when last_mc * sp_div <= n
    uint32_t sp_cooldown = 0;    // steps to stay dense after an abort
    uint32_t* d_bhist = nullptr; // byte-pair histogram of the first count (65,536 u32)
    uint32_t count_bytes_on = 1; // first count by the byte-pair histogram (0: hashed k_count_full)
    uint32_t lx_size_on = 1;     // word table sized from a sampled distinct count (0: from the word count)
    uint32_t seg8 = 1;           // zone segments of 8K symbols for zones <= 512K (GBPE_DEBUG seg8; 0: 16K)
    uint32_t zseg_lo = 8192;     // zones above this many symbols run as zone segments (GBPE_DEBUG zslo; 16384
                                 // = round 4: 1 GiB 0.557 vs 0.548 s, C2 equal, C1 11.6 vs 11.8 ms, profiles/r5/s30)
    uint32_t z256 = 0xFFFFFFFFu; // largest zone for the 256-thread k_body form (GBPE_DEBUG z256; 0: always 1024)
    uint32_t body_sub = 4;       // most k_body workgroups per bitmap word (1, 2, 4; GBPE_DEBUG bsub;
                                 // C1 13.5 -> 11.9 ms at 4, profiles/r5/s21)
    uint32_t body_min = 256;     // k_body workgroups at least, one bitmap word each at most (GBPE_DEBUG bmin;
                                 // 1 = the round-4 sizing of >= 16 / 32 words per workgroup)
    uint32_t lx_wg = 16384;      // k_lx_hash workgroups (at least LX_WPT words per thread; GBPE_DEBUG lxwg)
    bool lx_two = true;          // two-stage word-table build for large segments (GBPE_DEBUG lxtwo=0: one stage)
    uint32_t lx_resize = 0;      // builds whose sampled table was too small (rerun at full size)
    uint32_t lx_div = 16;        // with the lexicon: enter once next_mc * lx_div <= n, from the first step on (GBPE_DEBUG lxdiv)
    uint32_t sub_zone = 1u << 20;   // sparse steps run in sub-steps of sub_k merges while the zone exceeds this
    uint32_t sub_k = 16;            // (the zone shrinks between them; GBPE_DEBUG subz, subk)
    bool zone16 = true;             // u16 zones of 8K-16K symbols: the 16-per-thread zone pass 
    uint32_t sp_zt = 5;          // zone target = sp_zt * last_mc + 64 (>= zone_f; GBPE_DEBUG zt; 4/5/6/7 measured
                                 // 0.895/0.893/0.918/0.918 s at 1 GiB with zone_f 3)
    uint32_t shrink_pct = 200;   // shrink once the zone exceeds shrink_pct % of the target + 4096 
    uint32_t zone_f = 3;         // single-GPU zone rule factor (sel_inline, >= 3)
    uint32_t refresh_blocks = 0; // k_refresh grid (0 = 2 per CU)
    uint32_t refresh_late_z = 16384; // ... for zones of at most this many symbols
    uint32_t refresh_late = 64;  // k_refresh grid of late steps (0 = unchanged)
    bool rehash_on = true;       // grow the table inside the sparse loop (GBPE_DEBUG rehash=0: exit, grow, recount)
    uint32_t body_cap = 256;     // most k_body workgroups (one per CU)
    bool body_fit = true;        // the body's workgroups leave the zone's their CUs (GBPE_DEBUG bodyfit=0: off)
    bool pair_on = true;         // paired launches (GBPE_DEBUG pair=0: one merge per launch)
    bool pair_one = true;        // zones just above the zone_one form shrink into it (GBPE_DEBUG pone)
    double pair_rate = 0.5;      // second merges per launch of the last paired step (sizes the next step's launches)
    uint64_t pair_done = 0;      // merges run as the second of a launch (stats)
    uint32_t ptrace = 0;         // GBPE_DEBUG ptrace=1: every step's form and pairing on stderr
    uint32_t* d_clog = nullptr;  // GBPE_SPARSE_TRACE: per-merge candidate / hit sectors
    uint32_t* h_clog = nullptr;
    FILE* trace = nullptr;
    uint32_t htime = 0;          // GBPE_DEBUG htime=1: host enqueue / wait split of every step (stderr at destroy)
    double ht_enq = 0, ht_wait = 0, ht_enq_late = 0, ht_wait_late = 0, ht_pre = 0, ht_post = 0, ht_out = 0;
    double ht_shrink = 0, ht_filters = 0, ht_grow = 0;
    uint64_t ht_nshrink = 0, ht_nfilters = 0;
    std::chrono::steady_clock::time_point ht_last{};   // the previous step's return
    uint64_t ht_steps = 0, ht_steps_late = 0, ht_merges_late = 0;
    // word-lexicon body (lexicon.h): the sectors hold one copy of every
    // distinct body word instead of the body itself
    bool lex = false;            // the current sparse entry uses it
    bool lex_on = true;          // GBPE_DEBUG lexicon=0: never
    bool lex_only = false;       // built from shard lexicons (gbpe_trainer_create_from_lexicon): no dense stream,
                                 // the body's stream order lives on the ranks; never leaves the sparse loop
    void* lx_store = nullptr;    // distinct words, each followed by a 0 separator (S symbols)
    uint32_t* lx_mul = nullptr;  // per store symbol: its word's occurrences (0 = separator / padding)
    uint64_t lx_cap = 0, lx_len = 0;   // store symbols: capacity, used
    uint32_t* lx_occ = nullptr;  // body words in stream order: uid, or LX_LIT | symbol
    uint64_t lx_occ_cap = 0, lx_nocc = 0;
    uint32_t* lx_w0 = nullptr;   // first uid of each sector window
    uint32_t lx_nuid = 0, lx_uid_cap = 0;
    void* lx_tmp = nullptr;      // build / expansion scratch (grown, kept)
    uint64_t lx_tmp_bytes = 0;
    uint64_t lx_words = 0, lx_builds = 0, lx_fallbacks = 0;   // stats
};

namespace {

int tr_err(gbpe_trainer* t, int code, const char* msg) { return gbpe_set_error(t->ctx, code, "%s", msg); }

#define TR_HIP(t, call) GBPE_HIP((t)->ctx, call)

// the symbols the sparse kernels merge: the lexicon store, or the body sectors in place
inline void* sp_body(const gbpe_trainer* t) { return t->lex ? t->lx_store : t->buf[t->bcur]; }
inline uint32_t* sp_mul(const gbpe_trainer* t) { return t->lex ? t->lx_mul : nullptr; }
// the single-GPU selection's zone rule (sel_inline)
inline SelShard sel_single(const gbpe_trainer* t) {
    SelShard sh;
    sh.zf = t->zone_f;
    return sh;
}


uint32_t grid_persistent(const gbpe_ctx* ctx, uint64_t work_tiles, uint32_t per_cu) {
    uint64_t g = (uint64_t)(ctx->num_cu > 0 ? ctx->num_cu : 256) * per_cu;
    if (work_tiles < g) g = work_tiles;
    return (uint32_t)(g ? g : 1);
}
// a grid over argmax blocks: every workgroup owns at most 64 (one flag ballot)
uint32_t grid_blocks(const gbpe_ctx* ctx, uint32_t nblk, uint32_t per_cu) {
    return std::max<uint32_t>(grid_persistent(ctx, nblk, per_cu), (uint32_t)gbpe_div_up(nblk, 64));
}

// the partial maxima of the sparse selection (one per k_refresh workgroup), sized
// for the table's blocks (sparse entry; after every table resize)
int part_alloc(gbpe_trainer* t) {
    pool_free(t->ctx, t->part);
    t->part = nullptr;
    TR_HIP(t, pool_malloc(t->ctx, &t->part, 2ull * (t->tb.nblk + 1) * sizeof(uint64_t)));   // two keys per workgroup
    return GBPE_OK;
}

// new (empty) table arrays of 2^lg slots; the caller recounts (table_rebuild)
int table_resize(gbpe_trainer* t, uint32_t lg) {
    hipStream_t s = t->ctx->stream;
    TR_HIP(t, hipStreamSynchronize(s));
    pool_free(t->ctx, t->tb.slots);
    pool_free(t->ctx, t->tb.bmax);
    pool_free(t->ctx, t->tb.bmax2);
    pool_free(t->ctx, t->tb.dirty);
    pool_free(t->ctx, t->tb.dlist);
    pool_free(t->ctx, t->tb.blive);
    t->tb.slots = nullptr, t->tb.bmax = nullptr, t->tb.bmax2 = nullptr, t->tb.dirty = nullptr, t->tb.dlist = nullptr, t->tb.blive = nullptr;
    const uint64_t slots = 1ull << lg;
    t->table_log2 = lg;
    t->tb.mask = (uint32_t)(slots - 1);
    t->tb.nblk = (uint32_t)(slots >> BLK_LOG2);
    if (pool_malloc(t->ctx, &t->tb.slots, slots * sizeof(uint2)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.bmax, t->tb.nblk * sizeof(uint64_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.bmax2, t->tb.nblk * sizeof(uint64_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.dirty, t->tb.nblk * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.dlist, (t->tb.nblk + 1) * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.blive, t->tb.nblk * sizeof(uint32_t)) != hipSuccess)
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(pair table, 2^%u slots) failed", lg);
    TR_HIP(t, hipMemsetAsync(t->tb.dirty, 0, t->tb.nblk * sizeof(uint32_t), s));
    t->g_refresh = grid_blocks(t->ctx, t->tb.nblk, 2);
    if (t->refresh_blocks) t->g_refresh = std::max<uint32_t>(t->refresh_blocks, (uint32_t)gbpe_div_up(t->tb.nblk, 64));
    if (t->part) return part_alloc(t);   // one partial maximum per k_refresh workgroup
    return GBPE_OK;
}

// bytes_only: every symbol is a byte (the stream as trainer creation builds it)
int table_rebuild(gbpe_trainer* t, bool bytes_only = false) {
    hipStream_t s = t->ctx->stream;
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    TR_HIP(t, hipMemsetAsync(t->tb.slots, 0, slots * sizeof(uint2), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax2, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.blive, 0, (uint64_t)t->tb.nblk * sizeof(uint32_t), s));
    TR_HIP(t, hipMemsetAsync(&t->st->used, 0, sizeof(uint32_t), s));
    const uint64_t ntiles = gbpe_div_up(t->n, TILE);
    const uint32_t g = grid_persistent(t->ctx, ntiles, 2);
    if (bytes_only && t->count_bytes_on) {
        if (!t->d_bhist && pool_malloc(t->ctx, (void**)&t->d_bhist, 65536 * sizeof(uint32_t)) != hipSuccess) {
            t->d_bhist = nullptr;
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(byte-pair histogram) failed");
        }
        uint32_t* gh = t->d_bhist;
        TR_HIP(t, hipMemsetAsync(gh, 0, 65536 * sizeof(uint32_t), s));
        const uint64_t ncu = t->ctx->num_cu > 0 ? (uint64_t)t->ctx->num_cu : 256u;
        const uint32_t gb = 2u * (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ncu, gbpe_div_up(t->n, 16ull * CB_T)));
        if (t->u16)
            hipLaunchKernelGGL(k_count_bytes<uint16_t>, dim3(gb), dim3(CB_T), 0, s, (const uint16_t*)t->buf[t->cur],
                               (uint64_t)t->n, gh);
        else
            hipLaunchKernelGGL(k_count_bytes<uint32_t>, dim3(gb), dim3(CB_T), 0, s, (const uint32_t*)t->buf[t->cur],
                               (uint64_t)t->n, gh);
        hipLaunchKernelGGL(k_count_hist, dim3(256), dim3(256), 0, s, (const uint32_t*)gh, t->st, t->tb);
        GBPE_LAUNCH_CHECK(t->ctx);
    } else if (t->u16)
        hipLaunchKernelGGL(k_count_full<uint16_t>, dim3(g), dim3(TPB), 0, s, t->st,
                           (const uint16_t*)t->buf[t->cur], t->tb);
    else
        hipLaunchKernelGGL(k_count_full<uint32_t>, dim3(g), dim3(TPB), 0, s, t->st,
                           (const uint32_t*)t->buf[t->cur], t->tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    hipLaunchKernelGGL(k_clear_dirty_all, dim3(gbpe_div_up(t->tb.nblk, 256)), dim3(256), 0, s, t->st, t->tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    if (t->u16)
        hipLaunchKernelGGL(k_refresh<uint16_t>, dim3(grid_blocks(t->ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st, 0u,
                           0, t->tb, (uint16_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    else
        hipLaunchKernelGGL(k_refresh<uint32_t>, dim3(grid_blocks(t->ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st, 0u,
                           0, t->tb, (uint32_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

// Growing the table inside the sector-sparse loop: every count in the table is
// exact between steps (the body's multiplicities included), so the live entries
// move to the larger table as they are — no exit to one dense stream, no recount
// and no lexicon rebuild on re-entry (C5 grew 2^20 -> 2^25 in five such exits).
__global__ __launch_bounds__(TPB) void k_rehash(const uint2* __restrict__ old, uint64_t nold, DevState* st, Table tb) {
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i < nold; i += (uint64_t)gridDim.x * TPB) {
        const uint2 e = old[i];
        if (e.x && (int32_t)e.y > 0) table_add(tb, st, e.x, e.y);
    }
}

int table_rehash(gbpe_trainer* t, uint32_t lg) {
    hipStream_t s = t->ctx->stream;
    uint2* old = t->tb.slots;
    const uint64_t nold = (uint64_t)t->tb.mask + 1;
    t->tb.slots = nullptr;   // kept until the live entries have moved
    int rc = table_resize(t, lg);
    if (rc != GBPE_OK) {
        pool_free(t->ctx, old);
        return rc;
    }
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    TR_HIP(t, hipMemsetAsync(t->tb.slots, 0, slots * sizeof(uint2), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax2, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.blive, 0, (uint64_t)t->tb.nblk * sizeof(uint32_t), s));
    TR_HIP(t, hipMemsetAsync(&t->st->used, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_rehash, dim3(grid_persistent(t->ctx, gbpe_div_up(nold, TPB), 4)), dim3(TPB), 0, s,
                       (const uint2*)old, nold, t->st, t->tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    hipLaunchKernelGGL(k_clear_dirty_all, dim3(gbpe_div_up(t->tb.nblk, 256)), dim3(256), 0, s, t->st, t->tb);
    // block maxima and the per-workgroup partial maxima the next selection reads
    if (t->u16)
        GBPE_LAUNCH_REFRESH(uint16_t, t->g_refresh, t->tb.nblk, s, t->st, 0u, 0, t->tb, (uint16_t*)nullptr,
                            (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(), t->part,
                            (uint32_t*)nullptr);
    else
        GBPE_LAUNCH_REFRESH(uint32_t, t->g_refresh, t->tb.nblk, s, t->st, 0u, 0, t->tb, (uint32_t*)nullptr,
                            (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(), t->part,
                            (uint32_t*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    TR_HIP(t, hipStreamSynchronize(s));
    pool_free(t->ctx, old);
    return GBPE_OK;
}

template <typename S>
int launch_merge(gbpe_trainer* t, uint32_t round, hipStream_t s, uint32_t g_delta, uint32_t g_compact,
                 uint32_t g_refresh, bool timing, hipEvent_t* ev) {
    S* cur = (S*)t->buf[t->cur ^ (round & 1)];
    S* oth = (S*)t->buf[t->cur ^ (round & 1) ^ 1];
    const bool exact = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) != 0;
    if (timing) TR_HIP(t, hipEventRecord(ev[0], s));
    hipLaunchKernelGGL(k_select, dim3(1), dim3(SEL_THREADS), 0, s, t->st, t->tb, t->d_log, t->grpsum,
                       (DevState*)nullptr, exact ? 1u : 0u);
    if (timing) TR_HIP(t, hipEventRecord(ev[1], s));
    // many tiles: TPW tiles per k_delta workgroup (fewer hot-pair flushes)
    const bool mt = t->delta_mt && g_delta >= t->delta_mt;
    const uint32_t tpw = t->delta_tpw;
    const uint32_t g_mt = (uint32_t)gbpe_div_up(g_delta, tpw);
    // stale-tail blocks (reference compaction): ~2K symbols each of the largest
    // possible tail (n/2), at most 1024
    const uint32_t g_mtail = exact ? 0u : (uint32_t)std::min<uint64_t>(1024, gbpe_div_up((uint64_t)t->n / 2 + 1, 2048));
    // the single-tile k_delta's tail blocks (1024-slot LDS table: ~1K-symbol slices)
    const uint32_t g_dtail = exact ? 0u : (uint32_t)std::min<uint64_t>(1024, gbpe_div_up((uint64_t)t->n / 2 + 1, 1024));
    if (exact) {
        if (mt)
            hipLaunchKernelGGL(tpw == 32 ? (k_delta_mt<S, true, 32>) : tpw == 16 ? (k_delta_mt<S, true, 16>) : (k_delta_mt<S, true, 8>),
                               dim3(g_mt + g_mtail), dim3(TPB), 0, s, t->st, round, (const S*)cur, t->tb, t->hitmask,
                               t->tile_cnt, t->grpsum, g_delta, g_mt, 0u, ZdrView());
        else
            hipLaunchKernelGGL((k_delta<S, true>), dim3(g_delta), dim3(TPB), 0, s, t->st, round, (const S*)cur, t->tb,
                               t->hitmask, t->tile_cnt, t->grpsum, g_delta, 0xFFFFFFFFu);
        if (timing) TR_HIP(t, hipEventRecord(ev[3], s));
        hipLaunchKernelGGL((k_compact<S, true>), dim3(g_compact), dim3(CTPB), 0, s, t->st, round, cur, oth,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb);
    } else {
        if (mt)
            hipLaunchKernelGGL(tpw == 32 ? (k_delta_mt<S, false, 32>) : tpw == 16 ? (k_delta_mt<S, false, 16>) : (k_delta_mt<S, false, 8>),
                               dim3(g_mt + g_mtail), dim3(TPB), 0, s, t->st, round, (const S*)cur, t->tb, t->hitmask,
                               t->tile_cnt, t->grpsum, g_delta, g_mt, 0u, ZdrView());
        else
            hipLaunchKernelGGL((k_delta<S, false>), dim3(g_delta + g_dtail), dim3(TPB), 0, s, t->st, round, (const S*)cur,
                               t->tb, t->hitmask, t->tile_cnt, t->grpsum, g_delta, g_delta);
        if (timing) TR_HIP(t, hipEventRecord(ev[3], s));
        hipLaunchKernelGGL((k_compact<S, false>), dim3(g_compact), dim3(CTPB), 0, s, t->st, round, cur, oth,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb);
    }
    if (timing) TR_HIP(t, hipEventRecord(ev[2], s));
    FusedSel fs;
    fs.log = nullptr;
    fs.grpsum = t->grpsum;
    fs.exact = exact ? 1u : 0u;
    GBPE_LAUNCH_REFRESH(S, g_refresh, t->tb.nblk, s, t->st, round, 1, t->tb, cur, (const uint32_t*)nullptr,
                        (DevState*)nullptr, (uint32_t*)nullptr, fs, (uint64_t*)nullptr, (uint32_t*)nullptr);
    if (timing) TR_HIP(t, hipEventRecord(ev[4], s));
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

// ── sector-sparse loop: launches and re-layouts ──

struct SpGrid {
    uint32_t body, copy, zdelta, zcompact, refresh;
    uint32_t wpg = 16;    // bitmap words per k_body workgroup
    uint32_t sub = 1;     // k_body workgroups per bitmap word (wpg = 1)
    bool seg8 = false;    // zone segments of 8K symbols (1024 threads x 8), else 16K
    uint32_t ztail = 0;   // stale-tail slice blocks of the multi-tile zone k_delta
    uint32_t zone1;   // zone workgroups inside k_body: 1 = zone_one, >= 2 = zone_seg segments, 0 = multi-tile passes
    int bt;       // k_body workgroup size (256 or 1024)
    bool pair = false;   // launches may run two merges (zone_one in the 256-thread form)
};

template <typename S>
uint32_t zone_max(int bt) {
    return bt == 1023 ? 1024u * 16u : bt == 1024 ? ZoneDim<S, 1024>::ZMAX : ZoneDim<S, 256>::ZMAX;
}
// k_body grid: bitmap words per workgroup (>= the measured best 16 / 32 at C2 size),
// at most `cap` workgroups (default: body_cap, one per CU)
inline void body_grid(const gbpe_trainer* t, int bt, uint32_t* nbody, uint32_t* wpg, uint32_t cap = 0,
                      uint32_t* sub = nullptr) {
    const uint32_t W = (uint32_t)gbpe_div_up(t->nsec, 32);
    const uint32_t minw = bt == 1024 ? 32u : 16u;
    uint32_t g = (uint32_t)gbpe_div_up(W, minw);
    // but at least body_min workgroups (one bitmap word, 32 sectors, each at least):
    // a word's candidates then spread over more CUs instead of queueing on one
    // workgroup's waves (round 5, profiles/r5/s20: bmin 1 -> 256 took C1 25.1 ->
    // 13.2 ms, C2 0.470 -> 0.428 s, 1 GiB 0.602 -> 0.568 s; C5 unchanged — its
    // 131K-sector bitmap rows already fill every CU)
    const uint32_t gmin = std::min<uint32_t>(W, t->body_min);
    if (g < gmin) g = gmin;
    if (g > (cap ? cap : t->body_cap)) g = cap ? cap : t->body_cap;
    if (g == 0) g = 1;
    *wpg = (uint32_t)gbpe_div_up(W, g);
    if (*wpg == 0) *wpg = 1;
    *nbody = (uint32_t)gbpe_div_up(W, *wpg);
    if (*nbody == 0) *nbody = 1;
    if (sub) {   // a row of few words: 2 or 4 workgroups per word (slices of 16 / 8 sectors)
        *sub = 1;
        const uint32_t c = cap ? cap : t->body_cap;
        while (*sub * 2 <= t->body_sub && (uint64_t)W * *sub * 2 <= c) *sub *= 2;
        if (*sub > 1) {
            *wpg = 1;
            *nbody = W * *sub;
        }
    }
}

// launch k_body<S, EXACT, bt> (one instantiation per workgroup size)
// bt: 256, 1024, or 1023 = 1024 threads with 16 zone symbols each (u16 zones of
// 8K-16K symbols: half the per-thread zone work of the 32K form; 1 GiB en1g
// 1.017 -> 0.963 s.  1024 threads x 8 for zones <= 8K instead of 256 x 32 was
// slower: C2 0.66 vs 0.61 s)
template <typename S, bool EXACT, typename... A>
void launch_body(int bt, uint32_t grid, hipStream_t s, A... args) {
    if (bt == 2048)   // zone segments inside k_body (the ZSEG form, 1024 threads)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024, 16, true>), dim3(grid), dim3(1024), 0, s, args...);
    else if (bt == 2049)   // ... with 8K-symbol segments (zones <= 512K)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024, 8, true>), dim3(grid), dim3(1024), 0, s, args...);
    else if (bt == 1023 && sizeof(S) == 2)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024, 16>), dim3(grid), dim3(1024), 0, s, args...);
    else if (bt >= 1023)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024>), dim3(grid), dim3(1024), 0, s, args...);
    else
        hipLaunchKernelGGL((k_body<S, EXACT, 256>), dim3(grid), dim3(256), 0, s, args...);
}

template <typename S>
int launch_merge_sparse(gbpe_trainer* t, uint32_t round, hipStream_t s, const SpGrid& g, bool timing, hipEvent_t* ev) {
    S* zc = (S*)t->zbuf[t->zcur ^ (round & 1)];
    S* zo = (S*)t->zbuf[t->zcur ^ (round & 1) ^ 1];
    const bool exact = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) != 0;
    if (timing) TR_HIP(t, hipEventRecord(ev[0], s));
    if (timing) TR_HIP(t, hipEventRecord(ev[1], s));   // selection runs inside k_body (sel_inline)
    // zone segments run inside k_body (its ZSEG form)
    const bool inbody = g.zone1 >= 2;
    const uint32_t gb = g.body + (g.zone1 ? g.zone1 : g.copy);
    const uint32_t z1 = g.zone1;   // k_body's own zone workgroups
    const int bt = inbody ? (g.seg8 ? 2049 : 2048) : g.bt;
    SelShard sh = sel_single(t);
    sh.sub = g.sub;
    sh.k2 = g.pair ? 1u : 0u;
    if ((uint64_t)g.body + 1 > t->wg_cap)   // k_body's per-workgroup byte counters (and the zone's after them)
        return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "k_body grid (%u) above its byte counters (%llu)", g.body,
                              (unsigned long long)t->wg_cap);
    // events: [1] k_body [3] zone k_delta + k_compact (multi-tile zone) [2] k_refresh [4]
    // k_body picks the zone buffers by the state's merge index (a paired launch runs two
    // merges); the multi-tile kernels below run one merge per launch, so round = index
    S* zb0 = (S*)t->zbuf[t->zcur];
    S* zb1 = (S*)t->zbuf[t->zcur ^ 1];
    if (exact)
        launch_body<S, true>(bt, gb, s, t->st, round, (S*)sp_body(t), t->sec, t->bits, t->W, g.wpg, t->sig, t->tb,
                             g.body, zb1, (S*)t->wtmp, t->d_clog ? 1u : 0u, t->zst, zb0, z1,
                             (const uint64_t*)t->part, g.refresh, t->d_log, t->grpsum, t->wg_bytes, t->tb, sh,
                             sp_mul(t), (ZSegState*)t->zseg);
    else
        launch_body<S, false>(bt, gb, s, t->st, round, (S*)sp_body(t), t->sec, t->bits, t->W, g.wpg, t->sig, t->tb,
                              g.body, zb1, (S*)t->wtmp, t->d_clog ? 1u : 0u, t->zst, zb0, z1,
                              (const uint64_t*)t->part, g.refresh, t->d_log, t->grpsum, t->wg_bytes, t->tb, sh,
                              sp_mul(t), (ZSegState*)t->zseg);
    if (timing) TR_HIP(t, hipEventRecord(ev[3], s));
    if (!g.zone1 && !exact && t->zdr_on && t->zdr_out) {
        // a zone of many tiles, reference compaction: tiles dump their deltas, k_churn
        // runs the stale window and tail, k_zdr adds each distinct pair once (train_dev.h)
        const bool mt = t->delta_mt && g.zdelta >= t->delta_mt;
        const uint32_t g_mt = (uint32_t)gbpe_div_up(g.zdelta, 8);
        const uint32_t ntw = mt ? g_mt : g.zdelta;
        const uint32_t gch = (uint32_t)std::min<uint64_t>(ZDR_P, std::max<uint64_t>(1, gbpe_div_up(((uint32_t)t->n - t->h_st->B) / 5 + 1, 16384)));
        ZdrView zv;
        zv.out = t->zdr_out;
        zv.offs = t->zdr_offs;
        zv.flag = t->zdr_flag;
        zv.ntile = ntw;
        zv.tag = (uint32_t)(t->done + round + 1);
        if (ntw > t->zdr_ntile) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "zone delta dumps too small");
        if (mt)
            hipLaunchKernelGGL((k_delta_mt<S, false, 8>), dim3(g_mt), dim3(TPB), 0, s, t->zst, round, (const S*)zc, t->tb,
                               t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g_mt, 0u, zv);
        else
            hipLaunchKernelGGL((k_delta<S, false, true>), dim3(g.zdelta), dim3(TPB), 0, s, t->zst, round, (const S*)zc,
                               t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g.zdelta, zv);
        hipLaunchKernelGGL((k_compact<S, false, true>), dim3(g.zdelta), dim3(CTPB), 0, s, t->zst, round, zc, zo,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb,
                           (const S*)t->wtmp, (const DevState*)t->st, 1u);
        hipLaunchKernelGGL(k_churn<S>, dim3(gch), dim3(CH_BT), 0, s, t->zst, round, zc, zo, (const uint32_t*)t->hitmask,
                           (const uint32_t*)t->grpsum, (const S*)t->wtmp, t->tb, zv, ntw);
        hipLaunchKernelGGL(k_zdr, dim3(ZDR_P), dim3(TPB), 0, s, zv, ntw + gch, t->tb, t->zst, round);
    } else if (!g.zone1) {
        // a zone of many tiles (the lexicon loop's first merges): TPW tiles per
        // workgroup and one flush of their hot pairs, as in the dense loop
        const bool mt = t->delta_mt && g.zdelta >= t->delta_mt;
        const uint32_t g_mt = (uint32_t)gbpe_div_up(g.zdelta, 8);
        if (exact && mt)
            hipLaunchKernelGGL((k_delta_mt<S, true, 8>), dim3(g_mt), dim3(TPB), 0, s, t->zst, round, (const S*)zc, t->tb,
                               t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g_mt);
        else if (mt)
            hipLaunchKernelGGL((k_delta_mt<S, false, 8>), dim3(g_mt + g.ztail), dim3(TPB), 0, s, t->zst, round,
                               (const S*)zc, t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g_mt);
        else if (exact)
            hipLaunchKernelGGL((k_delta<S, true, true>), dim3(g.zdelta), dim3(TPB), 0, s, t->zst, round, (const S*)zc,
                               t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, 0xFFFFFFFFu);
        else   // + stale-tail slice blocks: the zone's tail (<= mc <= zone/5) in ~2K-symbol slices
            hipLaunchKernelGGL((k_delta<S, false, true>), dim3(g.zdelta + g.ztail), dim3(TPB), 0, s, t->zst, round,
                               (const S*)zc, t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g.zdelta);
    }
    if (!g.zone1 && !(!exact && t->zdr_on && t->zdr_out)) {
        if (exact)
            hipLaunchKernelGGL((k_compact<S, true, true>), dim3(g.zcompact), dim3(CTPB), 0, s, t->zst, round, zc, zo,
                               (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum,
                               t->tb, (const S*)t->wtmp, (const DevState*)t->st);
        else
            hipLaunchKernelGGL((k_compact<S, false, true>), dim3(g.zcompact), dim3(CTPB), 0, s, t->zst, round, zc, zo,
                               (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum,
                               t->tb, (const S*)t->wtmp, (const DevState*)t->st);
    }
    if (timing) TR_HIP(t, hipEventRecord(ev[2], s));
    GBPE_LAUNCH_REFRESH(S, g.refresh, t->tb.nblk, s, t->st, round, 2, t->tb, (S*)nullptr, (const uint32_t*)nullptr,
                        t->zst, t->d_clog, FusedSel(), t->part, t->zseg);
    if (timing) TR_HIP(t, hipEventRecord(ev[4], s));
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

template <typename T>
int sp_grow(gbpe_trainer* t, T** p, uint64_t* cap, uint64_t need) {
    if (*p && *cap >= need) return GBPE_OK;
    pool_free(t->ctx, *p);
    *p = nullptr;
    *cap = 0;
    if (pool_malloc(t->ctx, (void**)p, need * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(sparse layout, %llu B) failed",
                              (unsigned long long)(need * sizeof(T)));
    }
    *cap = need;
    return GBPE_OK;
}

// the token bitmap's rows at a new stride (bits of sectors past the old width: 0)
__global__ void k_restride(const uint32_t* __restrict__ old, uint32_t w_old, uint32_t* __restrict__ nb, uint32_t w_new,
                           uint64_t rows) {
    const uint64_t tot = rows * w_new;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = i / w_new, w = i % w_new;
        nb[i] = w < w_old ? old[r * w_old + w] : 0u;
    }
}

// grow-and-copy a device array to `want` elements (the first `keep` kept)
template <typename T>
int sp_regrow(gbpe_trainer* t, T** p, uint64_t* cap, uint64_t want, uint64_t keep) {
    if (*p && *cap >= want) return GBPE_OK;
    T* nb = nullptr;
    if (pool_malloc(t->ctx, (void**)&nb, want * sizeof(T)) != hipSuccess)
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(sparse layout growth, %llu B) failed",
                              (unsigned long long)(want * sizeof(T)));
    hipStream_t s = t->ctx->stream;
    if (*p && keep) TR_HIP(t, hipMemcpyAsync(nb, *p, keep * sizeof(T), hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    pool_free(t->ctx, *p);
    *p = nb;
    *cap = want;
    return GBPE_OK;
}

// Room for `need_sec` sectors, `need_store` lexicon store symbols and `need_occ`
// occurrences, growing by >= 1.5x with the contents kept (the token bitmap
// re-strided): the layout starts near its first build's size instead of the
// worst case of every zone shrink (C4's hand-over root: 64 GB of bitmap)
int sp_reserve(gbpe_trainer* t, uint64_t need_sec, uint64_t need_store, uint64_t need_occ) {
    hipStream_t s = t->ctx->stream;
    if (need_sec > t->nsec_cap || need_sec > (uint64_t)t->W * 32 || need_sec * SP_SIGW > t->sig_cap ||
        need_sec > t->loc_cap) {
        uint64_t cap = std::max<uint64_t>(need_sec, t->nsec_cap + t->nsec_cap / 2);
        cap = (cap + 31) & ~31ull;
        const uint64_t keep = t->nsec;
        int rc = sp_regrow(t, &t->sec, &t->nsec_cap, cap, keep);
        if (rc == GBPE_OK) rc = sp_regrow(t, &t->sig, &t->sig_cap, cap * SP_SIGW, keep * SP_SIGW);
        if (rc == GBPE_OK && t->lx_w0) {
            uint64_t wcap = 0;   // (allocated with the sector capacity)
            rc = sp_regrow(t, &t->lx_w0, &wcap, cap, keep);
        }
        if (rc != GBPE_OK) return rc;
        if (keep * SP_SIGW < cap * SP_SIGW)
            TR_HIP(t, hipMemsetAsync(t->sig + keep * SP_SIGW, 0, (cap - keep) * SP_SIGW * 4, s));
        pool_free(t->ctx, t->sp_loc);
        pool_free(t->ctx, t->sp_blk);
        t->sp_loc = nullptr;
        t->sp_blk = nullptr;
        t->loc_cap = 0;
        if (pool_malloc(t->ctx, &t->sp_loc, cap * 4) != hipSuccess ||
            pool_malloc(t->ctx, &t->sp_blk, (gbpe_div_up(cap, SCAN_BLK) + 1) * 8) != hipSuccess)
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(sector scratch) failed");
        t->loc_cap = cap;
        const uint32_t w_new = (uint32_t)gbpe_div_up(cap, 32);
        if (w_new > t->W || !t->bits) {
            uint32_t* nb = nullptr;
            const uint64_t words = (uint64_t)t->max_id * w_new;
            if (pool_malloc(t->ctx, &nb, words * 4) != hipSuccess)
                return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(token bitmap, %llu B) failed",
                                      (unsigned long long)(words * 4));
            if (t->bits && t->W)
                hipLaunchKernelGGL(k_restride, dim3(grid_persistent(t->ctx, gbpe_div_up(words, 256), 8)), dim3(256), 0, s,
                                   (const uint32_t*)t->bits, t->W, nb, w_new, (uint64_t)t->max_id);
            else
                TR_HIP(t, hipMemsetAsync(nb, 0, words * 4, s));
            GBPE_LAUNCH_CHECK(t->ctx);
            TR_HIP(t, hipStreamSynchronize(s));
            pool_free(t->ctx, t->bits);
            t->bits = nb;
            t->bits_cap = words;
            t->W = w_new;
        }
        // one byte counter per k_body workgroup (at most body_cap of them: body_grid) + the zone's
        const uint64_t wneed = std::max<uint64_t>(gbpe_div_up(w_new, SP_WPW_MIN), t->body_cap) + 2;
        if (t->wg_bytes && wneed > t->wg_cap) {
            uint64_t* nb = nullptr;
            TR_HIP(t, pool_malloc(t->ctx, &nb, wneed * sizeof(uint64_t)));
            TR_HIP(t, hipMemsetAsync(nb, 0, wneed * sizeof(uint64_t), s));
            TR_HIP(t, hipMemcpyAsync(nb, t->wg_bytes, t->wg_cap * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
            TR_HIP(t, hipStreamSynchronize(s));
            pool_free(t->ctx, t->wg_bytes);
            t->wg_bytes = nb;
            t->wg_cap = wneed;
        }
    }
    if (t->lx_store && need_store > t->lx_cap) {
        const uint64_t want = std::max<uint64_t>(need_store, t->lx_cap + t->lx_cap / 2);
        uint64_t c1 = t->lx_cap, c2 = t->lx_cap;
        void* st = t->lx_store;
        if (pool_malloc(t->ctx, &t->lx_store, want * t->bps) != hipSuccess) {
            t->lx_store = st;
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(word lexicon growth) failed");
        }
        TR_HIP(t, hipMemcpyAsync(t->lx_store, st, t->lx_len * t->bps, hipMemcpyDeviceToDevice, s));
        TR_HIP(t, hipStreamSynchronize(s));
        pool_free(t->ctx, st);
        int rc = sp_regrow(t, &t->lx_mul, &c1, want, t->lx_len);
        if (rc != GBPE_OK) return rc;
        (void)c2;
        t->lx_cap = want;
    }
    if (t->lx_occ && need_occ > t->lx_occ_cap) {
        const uint64_t want = std::max<uint64_t>(need_occ, t->lx_occ_cap + t->lx_occ_cap / 2);
        int rc = sp_regrow(t, &t->lx_occ, &t->lx_occ_cap, want, t->lx_nocc);
        if (rc != GBPE_OK) return rc;
    }
    return GBPE_OK;
}

// sectors over body positions [base, base + len) appended after sector t->nsec
// (their token bits and signatures too); base is a word start
template <typename S>
int sp_add_sectors(gbpe_trainer* t, uint32_t base, uint32_t len) {
    hipStream_t s = t->ctx->stream;
    const uint32_t nw = (uint32_t)gbpe_div_up(len, t->sp_secw);
    {
        int rc = sp_reserve(t, (uint64_t)t->nsec + nw, 0, 0);
        if (rc != GBPE_OK) return rc;
    }
    const S* body = (const S*)t->buf[t->bcur];
    hipLaunchKernelGGL(k_sp_sectors<S>, dim3((uint32_t)gbpe_div_up(nw, TPB / 64)), dim3(TPB), 0, s, body, base, len,
                       t->sp_secw, t->sp_loc, nw);
    hipLaunchKernelGGL(k_sp_sector_len, dim3((uint32_t)gbpe_div_up(nw, 256)), dim3(256), 0, s, (const uint32_t*)t->sp_loc,
                       nw, base + len, t->sec + t->nsec);
    if (t->nsec == 0) {   // a fresh build (sp_enter): whole columns
        hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(nw, TPB / 64)), dim3(TPB), 0, s, body,
                           (const uint2*)t->sec, 0u, nw, (uint32_t*)nullptr, t->W, t->sig);
        hipLaunchKernelGGL(k_sp_colbits<S>, dim3((uint32_t)gbpe_div_up(nw, 32)), dim3(TPB), 0, s, body,
                           (const uint2*)t->sec, nw, t->bits, t->W);
    } else {
        hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(nw, TPB / 64)), dim3(TPB), 0, s, body,
                           (const uint2*)t->sec, t->nsec, nw, t->bits, t->W, t->sig);
    }
    GBPE_LAUNCH_CHECK(t->ctx);
    t->nsec += nw;
    t->bend = base + len;
    return GBPE_OK;
}

// (re)build the pair signatures (and, with `with_bits`, the token bitmap) from the
// body sectors: stale entries make the filters looser, never wrong
template <typename S>
int sp_filters(gbpe_trainer* t, bool with_bits) {
    hipStream_t s = t->ctx->stream;
    hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(t->nsec, TPB / 64)), dim3(TPB), 0, s,
                       (const S*)sp_body(t), (const uint2*)t->sec, 0u, t->nsec, (uint32_t*)nullptr, t->W, t->sig);
    if (with_bits) {
        TR_HIP(t, hipMemsetAsync(t->bits, 0, (uint64_t)t->max_id * t->W * 4, s));
        hipLaunchKernelGGL(k_sp_colbits<S>, dim3((uint32_t)gbpe_div_up(t->nsec, 32)), dim3(TPB), 0, s,
                           (const S*)sp_body(t), (const uint2*)t->sec, t->nsec, t->bits, t->W);
    }
    GBPE_LAUNCH_CHECK(t->ctx);
    t->sp_age = 0;
    if (with_bits) t->sp_bits_age = 0;
    return GBPE_OK;
}

// ── word-lexicon body ──

// bump allocation over the trainer's lexicon scratch
struct LxCarve {
    char* base;
    uint64_t used = 0;
    template <typename T>
    T* take(uint64_t n) {
        const uint64_t b = (used + 255) & ~255ull;
        used = b + n * sizeof(T);
        return reinterpret_cast<T*>(base + b);
    }
};

int lx_scratch(gbpe_trainer* t, uint64_t bytes) {
    if (t->lx_tmp && t->lx_tmp_bytes >= bytes) return GBPE_OK;
    TR_HIP(t, hipStreamSynchronize(t->ctx->stream));
    pool_free(t->ctx, t->lx_tmp);
    t->lx_tmp = nullptr;
    t->lx_tmp_bytes = 0;
    if (pool_malloc(t->ctx, &t->lx_tmp, bytes) != hipSuccess) {
        t->lx_tmp = nullptr;
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(lexicon scratch, %llu B) failed", (unsigned long long)bytes);
    }
    t->lx_tmp_bytes = bytes;
    return GBPE_OK;
}

// exclusive scan of n u32 counts in place (k_chunk_scan1/2); blk gets n/SCAN_BLK + 2
// entries, the total at blk[nblk]
inline void lx_scan(hipStream_t s, uint32_t* v, uint64_t n, uint64_t* blk) {
    const uint64_t nb = gbpe_div_up(n ? n : 1, SCAN_BLK);
    hipLaunchKernelGGL(k_chunk_scan1, dim3((uint32_t)nb), dim3(SCAN_TPB), 0, s, (const uint32_t*)v, n, v, blk);
    hipLaunchKernelGGL(k_chunk_scan2, dim3(1), dim3(SCAN_TPB), 0, s, blk, nb, blk + nb);
}

// What a segment's words would add to the lexicon (nothing is committed yet)
struct LxPlan {
    bool ok = false;
    uint32_t nw = 0, nshort = 0, nlong = 0, nu = 0, T = 0;   // words, distinct short / long, entries, store symbols
    uint32_t *wpos = nullptr, *usz = nullptr, *umul = nullptr, *urep = nullptr, *occ = nullptr, *upre = nullptr;
    uint64_t* ublk = nullptr;
};

// Dedup the words of seg[0, len) (a word starts at 0): word starts, the word
// table, entries (uids from t->lx_nuid) and the segment's occurrence list, in
// the scratch.  plan.ok = false when a hash collision or a full word table
// makes the segment unusable, or (fresh) the store would not be much smaller
// than the segment.
template <typename S>
int lx_analyze(gbpe_trainer* t, const S* seg, uint32_t len, bool fresh, LxPlan& lp, const uint32_t* wmul = nullptr) {
    hipStream_t s = t->ctx->stream;
    lp = LxPlan();
    if (len == 0) return GBPE_OK;
    const uint64_t ntiles = gbpe_div_up(len, TILE);
    // word count first (sizes the scratch); the tile counts live outside the
    // scratch, which may move, so k_lx_wpos uses them as they are
    uint32_t* tc = nullptr;
    uint64_t* tb = nullptr;
    auto tc_free = gbpe_scope_exit([&] {
        pool_free(t->ctx, tc);
        pool_free(t->ctx, tb);
    });
    TR_HIP(t, pool_malloc(t->ctx, &tc, (ntiles + 64) * 4));
    TR_HIP(t, pool_malloc(t->ctx, &tb, (ntiles / SCAN_BLK + 4) * 8));
    hipLaunchKernelGGL(k_lx_count<S>, dim3((uint32_t)ntiles), dim3(TPB), 0, s, seg, len, tc);
    lx_scan(s, tc, ntiles, tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    {
        uint64_t nw64 = 0;
        TR_HIP(t, hipMemcpyAsync(&nw64, tb + gbpe_div_up(ntiles, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
        lp.nw = (uint32_t)nw64;
    }
    const uint32_t nw = lp.nw;
    // word table: room for every word at half load (Pfull), but sized from the
    // distinct words of a sample when the segment is long — a table of the
    // distinct words stays in the caches, one of all words (2 GB at 1 GiB) does not
    uint64_t Pfull = 4096;
    while (Pfull < 2ull * nw && Pfull < (1ull << 27)) Pfull <<= 1;
    const uint64_t nbbf = gbpe_div_up(Pfull, LX_TB);
    // the two-stage build (k_lx_hash records + k_lx_fold) for a large segment: its
    // records (LX_LT per stage-1 workgroup) and bucket offsets / sizes
    const auto wpt_of = [&](uint64_t nh) {
        return (uint32_t)std::max<uint64_t>(LX_WPT, gbpe_div_up(nh, (uint64_t)TPB * t->lx_wg));
    };
    constexpr uint32_t LX2_T = 1024, LX2_LT = 8192, LX2_WPT = 16;   // the two-stage build's first stage
    const uint64_t nwg_max = gbpe_div_up(nw, (uint64_t)LX2_T * LX2_WPT);
    const bool two = t->lx_two && nw >= (1u << 20);
    const uint64_t need = 9ull * (nw + 64) * 4 + Pfull * 16 + (nbbf + 64) * 4 +
                          2 * (nbbf / SCAN_BLK + (uint64_t)nw / SCAN_BLK + 8) * 8 + 32 * 256 +
                          (two ? nwg_max * LX2_LT * sizeof(LxSlot) + 2 * nwg_max * 256 * 4 + 1024 : 0);
    int rc = lx_scratch(t, need);
    if (rc != GBPE_OK) return rc;
    LxCarve c{(char*)t->lx_tmp};
    lp.wpos = c.take<uint32_t>(nw + 1);
    uint32_t* otmp = c.take<uint32_t>(nw + 1);
    uint32_t* longs = c.take<uint32_t>(nw + 1);
    lp.usz = c.take<uint32_t>(nw + 1);
    lp.umul = c.take<uint32_t>(nw + 1);
    lp.urep = c.take<uint32_t>(nw + 1);
    lp.occ = c.take<uint32_t>(nw + 1);
    auto* wtab = c.take<LxSlot>(Pfull);
    uint32_t* bc = c.take<uint32_t>(nbbf);
    uint64_t* bb = c.take<uint64_t>(nbbf / SCAN_BLK + 4);
    lp.ublk = c.take<uint64_t>((uint64_t)nw / SCAN_BLK + 4);
    uint32_t* ctr = c.take<uint32_t>(8);
    LxSlot* rec = two ? c.take<LxSlot>(nwg_max * LX2_LT) : nullptr;
    uint32_t* bmeta = two ? c.take<uint32_t>(2 * nwg_max * 256) : nullptr;
    hipLaunchKernelGGL(k_lx_wpos<S>, dim3((uint32_t)ntiles), dim3(TPB), 0, s, seg, len, (const uint32_t*)tc,
                       (const uint64_t*)tb, lp.wpos);
    uint32_t h[4] = {0, 0, 0, 0};
    uint64_t nshort = 0;
    // hash the first `nh` words into a P-slot table; h = {long words, overflow}, nshort = distinct
    auto hash_pass = [&](uint64_t P, uint32_t nh) -> int {
        const uint64_t nbb = gbpe_div_up(P, LX_TB);
        TR_HIP(t, hipMemsetAsync(wtab, 0, P * sizeof(LxSlot), s));
        TR_HIP(t, hipMemsetAsync(ctr, 0, 32, s));
        if (nh) {
            const uint32_t maxp = P < Pfull ? 256u : LX_PROBES;   // an estimated table gives up early when short
            // two stages (the main pass of a large segment): P >= 2^20 slots make 256 slices
            const uint32_t nwg2 = (uint32_t)gbpe_div_up(nh, (uint64_t)LX2_T * LX2_WPT);
            if (two && P >= (1ull << 20) && nh >= (1u << 20) && nwg2 <= nwg_max) {
                hipLaunchKernelGGL((k_lx_hash<S, LX2_T, LX2_LT>), dim3(nwg2), dim3(LX2_T), 0, s, seg, len,
                                   (const uint32_t*)lp.wpos, nh, wtab, (uint32_t)P, otmp, longs, ctr, wmul, maxp, LX2_WPT,
                                   rec, bmeta, 256u, nwg2);
                hipLaunchKernelGGL(k_lx_fold, dim3(256), dim3(FOLD_T), 0, s, (const LxSlot*)rec, (const uint32_t*)bmeta,
                                   nwg2, 256u, wtab, (uint32_t)P, ctr, maxp, LX2_LT);
            } else {
                const uint32_t wpt = wpt_of(nh);
                hipLaunchKernelGGL(k_lx_hash<S>, dim3((uint32_t)gbpe_div_up(nh, (uint64_t)TPB * wpt)), dim3(TPB), 0, s, seg,
                                   len, (const uint32_t*)lp.wpos, nh, wtab, (uint32_t)P, otmp, longs, ctr, wmul, maxp, wpt);
            }
        }
        hipLaunchKernelGGL(k_lx_tabcount, dim3((uint32_t)nbb), dim3(TPB), 0, s, (const LxSlot*)wtab, (uint32_t)P, bc);
        lx_scan(s, bc, nbb, bb);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipMemcpyAsync(h, ctr, 8, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipMemcpyAsync(&nshort, bb + gbpe_div_up(nbb, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
        return GBPE_OK;
    };
    uint64_t P = Pfull;
    constexpr uint32_t LX_SAMPLE = 1u << 22;   // words of the sample
    if (nw > 4u * LX_SAMPLE && t->lx_size_on) {
        rc = hash_pass(2ull * LX_SAMPLE, LX_SAMPLE);
        if (rc != GBPE_OK) return rc;
        if (!h[1]) {   // distinct words grow slower than words (Heaps): D ~ d (nw / sample)^0.8, at <= 1/3 load
            const double D = (double)(nshort + h[0]) * pow((double)nw / LX_SAMPLE, 0.8);
            uint64_t Pe = 1ull << 20;
            while ((double)Pe < 3.0 * D && Pe < Pfull) Pe <<= 1;
            P = Pe;
        }
    }
    rc = hash_pass(P, nw);
    if (rc != GBPE_OK) return rc;
    if (h[1] && P < Pfull) {   // the estimate was short: the full-size table
        P = Pfull;
        ++t->lx_resize;
        rc = hash_pass(P, nw);
        if (rc != GBPE_OK) return rc;
    }
    const uint64_t nbb = gbpe_div_up(P, LX_TB);
    if (h[1]) return GBPE_OK;   // word table overflow: not usable
    lp.nshort = (uint32_t)nshort;
    lp.nlong = h[0];
    lp.nu = lp.nshort + lp.nlong;
    if ((uint64_t)t->lx_nuid + lp.nu >= LX_LONG) return GBPE_OK;
    hipLaunchKernelGGL(k_lx_tabuid, dim3((uint32_t)nbb), dim3(TPB), 0, s, wtab, (uint32_t)P, (const uint32_t*)bc, (const uint64_t*)bb, (const uint32_t*)lp.wpos, nw, len, lp.usz, lp.umul, lp.urep);
    if (lp.nlong)
        hipLaunchKernelGGL(k_lx_longs, dim3((uint32_t)gbpe_div_up(lp.nlong, 256)), dim3(256), 0, s, (const uint32_t*)longs,
                           (const uint32_t*)ctr, lp.nshort, (const uint32_t*)lp.wpos, nw, len, lp.usz, lp.umul, lp.urep,
                           wmul);
    // store offsets: exclusive scan of the entry sizes, in `longs` (k_lx_longs,
    // queued before on the same stream, has consumed it)
    uint32_t* upre = longs;
    TR_HIP(t, hipMemcpyAsync(upre, lp.usz, (uint64_t)lp.nu * 4, hipMemcpyDeviceToDevice, s));
    lx_scan(s, upre, lp.nu, lp.ublk);
    GBPE_LAUNCH_CHECK(t->ctx);
    uint64_t T = 0;
    TR_HIP(t, hipMemcpyAsync(&T, lp.ublk + gbpe_div_up(lp.nu ? lp.nu : 1, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (fresh && T * 2 > len) return GBPE_OK;   // not worth it: the store would be more than half the body
    if (nw) {
        // the entries' compact copy (the store's layout) for the occurrence check
        S* rstore = nullptr;
        auto rs_free = gbpe_scope_exit([&] { pool_free(t->ctx, rstore); });
        TR_HIP(t, pool_malloc(t->ctx, &rstore, (T + 1) * sizeof(S)));
        if (lp.nu)
            hipLaunchKernelGGL(k_lx_fill<S>, dim3((uint32_t)gbpe_div_up(lp.nu, 256)), dim3(256), 0, s, seg,
                               (const uint32_t*)lp.urep, (const uint32_t*)lp.usz, (const uint32_t*)lp.umul,
                               (const uint32_t*)upre, (const uint64_t*)lp.ublk, lp.nu, rstore, (uint32_t*)nullptr);
        hipLaunchKernelGGL(k_lx_occ<S>, dim3((uint32_t)gbpe_div_up(nw, 256)), dim3(256), 0, s, seg, (const uint32_t*)lp.wpos, nw,
                           len, (const uint32_t*)otmp, (const LxSlot*)wtab, (uint32_t)P, (const S*)rstore,
                           (const uint32_t*)upre, (const uint64_t*)lp.ublk, (const uint32_t*)lp.usz, lp.nshort,
                           t->lx_nuid, lp.occ, ctr);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipMemcpyAsync(h, ctr, 8, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
        if (h[1]) return GBPE_OK;   // a hash collision (or a word missing from the table)
    }
    lp.T = (uint32_t)T;
    lp.upre = upre;
    lp.ok = true;
    return GBPE_OK;
}

// Append a planned segment to the lexicon: store entries (window-aligned), their
// sector windows after t->nsec with token bits and signatures, occurrences after
// t->lx_nocc.  plan.ok = false (nothing changed) when the capacities cannot take it.
template <typename S>
int lx_commit(gbpe_trainer* t, LxPlan& lp, const S* seg, bool fresh, bool keep_occ = true) {
    hipStream_t s = t->ctx->stream;
    const uint32_t SEC = t->sp_secw;
    const uint64_t sbase = gbpe_div_up(t->lx_len, SEC) * SEC;
    const uint64_t nwin = gbpe_div_up(lp.T ? lp.T : 1, SEC);
    const uint64_t kb = sbase / SEC;
    {
        int rc = sp_reserve(t, kb + nwin, sbase + nwin * SEC, keep_occ ? t->lx_nocc + lp.nw : 0);
        if (rc != GBPE_OK) return rc;
    }
    S* store = (S*)t->lx_store;
    if (sbase > t->lx_len) {   // alignment padding: separators no sector covers
        TR_HIP(t, hipMemsetAsync(store + t->lx_len, 0, (sbase - t->lx_len) * sizeof(S), s));
        TR_HIP(t, hipMemsetAsync(t->lx_mul + t->lx_len, 0, (sbase - t->lx_len) * 4, s));
    }
    const uint32_t* upre = lp.upre;
    if (lp.nu) {
        hipLaunchKernelGGL(k_lx_fill<S>, dim3((uint32_t)gbpe_div_up(lp.nu, 256)), dim3(256), 0, s, seg,
                           (const uint32_t*)lp.urep, (const uint32_t*)lp.usz, (const uint32_t*)lp.umul, upre,
                           (const uint64_t*)lp.ublk, lp.nu, store + sbase, t->lx_mul + sbase);
        TR_HIP(t, hipMemsetAsync(t->sp_loc, 0xFF, nwin * 4, s));
        hipLaunchKernelGGL(k_lx_secstart, dim3((uint32_t)gbpe_div_up(lp.nu, 256)), dim3(256), 0, s, upre,
                           (const uint64_t*)lp.ublk, lp.nu, SEC, (uint32_t)sbase, t->lx_nuid, t->sp_loc, t->lx_w0 + kb);
        hipLaunchKernelGGL(k_sp_sector_len, dim3((uint32_t)gbpe_div_up(nwin, 256)), dim3(256), 0, s,
                           (const uint32_t*)t->sp_loc, (uint32_t)nwin, (uint32_t)(sbase + lp.T), t->sec + kb);
    } else {
        TR_HIP(t, hipMemsetAsync(t->sec + kb, 0, nwin * sizeof(uint2), s));
    }
    if (lp.nw && keep_occ)
        TR_HIP(t, hipMemcpyAsync(t->lx_occ + t->lx_nocc, lp.occ, (uint64_t)lp.nw * 4, hipMemcpyDeviceToDevice, s));
    // token bits and signatures of the new sectors (a fresh build: whole columns)
    hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(nwin, TPB / 64)), dim3(TPB), 0, s, (const S*)store,
                       (const uint2*)t->sec, (uint32_t)kb, (uint32_t)nwin, fresh ? (uint32_t*)nullptr : t->bits, t->W, t->sig);
    if (fresh)
        hipLaunchKernelGGL(k_sp_colbits<S>, dim3((uint32_t)gbpe_div_up(nwin, 32)), dim3(TPB), 0, s, (const S*)store,
                           (const uint2*)t->sec, (uint32_t)nwin, t->bits, t->W);
    GBPE_LAUNCH_CHECK(t->ctx);
    t->nsec = (uint32_t)(kb + nwin);
    t->lx_len = sbase + lp.T;
    if (keep_occ) t->lx_nocc += lp.nw;
    t->lx_nuid += lp.nu;
    t->lx_words += lp.nw;
    return GBPE_OK;
}

// lexicon → dense stream: every body word occurrence's current symbols, in
// stream order, to dst[0, B); returns the symbol total through *tot.  The sizes
// are checked before anything is written: an occurrence naming no entry, or a
// total above dst_cap symbols, fails (GBPE_E_INVALID) with dst untouched.
template <typename S>
int lx_expand(gbpe_trainer* t, S* dst, uint64_t dst_cap, uint64_t* tot, const uint32_t* occ = nullptr, uint64_t n_occ = 0) {
    // occ: another occurrence list over this store (the lexicon hand-over's rank lists)
    hipStream_t s = t->ctx->stream;
    if (!occ) occ = t->lx_occ, n_occ = t->lx_nocc;
    const uint64_t nu = t->lx_nuid, no = n_occ;
    int rc = lx_scratch(t, (2 * nu + no + 64) * 4 + (no / SCAN_BLK + 8) * 8 + 4096);
    if (rc != GBPE_OK) return rc;
    LxCarve c{(char*)t->lx_tmp};
    uint32_t* coff = c.take<uint32_t>(nu + 1);
    uint32_t* clen = c.take<uint32_t>(nu + 1);
    uint32_t* olen = c.take<uint32_t>(no + 1);
    uint64_t* oblk = c.take<uint64_t>(no / SCAN_BLK + 4);
    uint32_t* bad = c.take<uint32_t>(4);
    TR_HIP(t, hipMemsetAsync(bad, 0, 4, s));
    if (t->nsec)
        hipLaunchKernelGGL(k_lx_wordpos<S>, dim3((uint32_t)gbpe_div_up(t->nsec, TPB / 64)), dim3(TPB), 0, s,
                           (const S*)t->lx_store, (const uint2*)t->sec, t->nsec, (const uint32_t*)t->lx_w0, coff, clen);
    if (no)
        hipLaunchKernelGGL(k_lx_olen, dim3((uint32_t)gbpe_div_up(no, 256)), dim3(256), 0, s, occ, no,
                           (const uint32_t*)clen, olen, (uint32_t)nu, bad);
    lx_scan(s, olen, no, oblk);
    GBPE_LAUNCH_CHECK(t->ctx);
    uint64_t total = 0;
    uint32_t hbad = 0;
    TR_HIP(t, hipMemcpyAsync(&total, oblk + gbpe_div_up(no ? no : 1, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    *tot = total;
    if (hbad) return gbpe_set_error(t->ctx, GBPE_E_INVALID, "lexicon expand: an occurrence names no word entry");
    if (total > dst_cap)
        return gbpe_set_error(t->ctx, GBPE_E_INVALID, "lexicon expand: the occurrences hold %llu symbols, room for %llu",
                              (unsigned long long)total, (unsigned long long)dst_cap);
    if (no)
        hipLaunchKernelGGL(k_lx_expand<S>, dim3((uint32_t)gbpe_div_up(no, 256)), dim3(256), 0, s, occ, no,
                           (const uint32_t*)coff, (const uint32_t*)clen, (const S*)t->lx_store, (const uint32_t*)olen,
                           (const uint64_t*)oblk, dst, (uint32_t)nu);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

// diagnostic (GBPE_DEBUG lex_check=1): the lexicon right after a build expands back to the body
template <typename S>
int lx_check(gbpe_trainer* t, const S* cur, uint32_t Zs, const LxPlan& lp) {
    hipStream_t s = t->ctx->stream;
    int rc = GBPE_OK;
    S* chk = nullptr;
    TR_HIP(t, pool_malloc(t->ctx, &chk, ((uint64_t)Zs + 64) * sizeof(S)));
    uint64_t tot = 0;
    rc = lx_expand<S>(t, chk, (uint64_t)Zs + 64, &tot);
    std::vector<S> a(Zs), b(Zs);
    TR_HIP(t, hipStreamSynchronize(s));
    TR_HIP(t, hipMemcpy(a.data(), chk, (uint64_t)Zs * sizeof(S), hipMemcpyDeviceToHost));
    TR_HIP(t, hipMemcpy(b.data(), cur, (uint64_t)Zs * sizeof(S), hipMemcpyDeviceToHost));
    pool_free(t->ctx, chk);
    uint64_t bad = Zs;
    for (uint64_t i = 0; i < Zs; ++i)
        if (a[i] != b[i]) {
            bad = i;
            break;
        }
    std::vector<uint32_t> mm(lp.T);
    std::vector<S> ss(lp.T);
    TR_HIP(t, hipMemcpy(mm.data(), t->lx_mul, (uint64_t)lp.T * 4, hipMemcpyDeviceToHost));
    TR_HIP(t, hipMemcpy(ss.data(), t->lx_store, (uint64_t)lp.T * sizeof(S), hipMemcpyDeviceToHost));
    uint64_t wsum = 0, nz = 0, badm = 0;
    for (uint32_t i = 0; i < lp.T; ++i) {
        wsum += mm[i];
        if ((ss[i] == 0) != (mm[i] == 0)) ++badm;
    }
    for (uint32_t i = 0; i < Zs; ++i) nz += (b[i] & Sym<S>::TM) ? 1 : 0;
    fprintf(stderr, "[lex-check] Zs=%u words=%u distinct=%u+%u store=%u expanded=%llu first_diff=%llu "
            "mult_sum=%llu nonzero_body=%llu sep_mismatch=%llu\n", Zs, lp.nw,
            lp.nshort, lp.nlong, lp.T, (unsigned long long)tot, (unsigned long long)bad,
            (unsigned long long)wsum, (unsigned long long)nz, (unsigned long long)badm);
    return rc;
}

// ── sector-sparse layout: allocations shared by sp_enter and the lexicon
//    hand-over (gbpe_trainer_create_from_lexicon) ──

// sector arrays for `cap` sectors: extents, scratch, token bitmap (W words per
// row), pair signatures — bitmap and signatures zeroed
int sp_alloc_layout(gbpe_trainer* t, uint64_t cap) {
    hipStream_t s = t->ctx->stream;
    int rc = sp_grow(t, &t->sec, &t->nsec_cap, cap);
    if (rc == GBPE_OK && (!t->sp_loc || t->loc_cap < cap)) {
        pool_free(t->ctx, t->sp_loc);
        pool_free(t->ctx, t->sp_blk);
        t->sp_loc = nullptr;
        t->sp_blk = nullptr;
        t->loc_cap = 0;
        if (pool_malloc(t->ctx, &t->sp_loc, cap * 4) != hipSuccess ||
            pool_malloc(t->ctx, &t->sp_blk, (gbpe_div_up(cap, SCAN_BLK) + 1) * 8) != hipSuccess)
            rc = gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(sector scratch) failed");
        else
            t->loc_cap = cap;
    }
    if (rc != GBPE_OK) return rc;
    t->W = (uint32_t)gbpe_div_up(cap, 32);
    rc = sp_grow(t, &t->bits, &t->bits_cap, (uint64_t)t->max_id * t->W);
    if (rc == GBPE_OK) rc = sp_grow(t, &t->sig, &t->sig_cap, cap * SP_SIGW);
    if (rc != GBPE_OK) return rc;
    t->nsec = 0;
    TR_HIP(t, hipMemsetAsync(t->bits, 0, (uint64_t)t->max_id * t->W * 4, s));
    TR_HIP(t, hipMemsetAsync(t->sig, 0, cap * SP_SIGW * 4, s));
    return GBPE_OK;
}

// word-lexicon store for `cap` sectors of sp_secw symbols, occurrence list of `ocap`
int sp_alloc_lexicon(gbpe_trainer* t, uint64_t cap, uint64_t ocap) {
    const uint64_t scap = cap * t->sp_secw;
    if (!t->lx_store || t->lx_cap < scap) {
        pool_free(t->ctx, t->lx_store);
        pool_free(t->ctx, t->lx_mul);
        pool_free(t->ctx, t->lx_w0);
        t->lx_store = nullptr;
        t->lx_mul = t->lx_w0 = nullptr;
        t->lx_cap = 0;
        if (pool_malloc(t->ctx, &t->lx_store, scap * t->bps) != hipSuccess || pool_malloc(t->ctx, &t->lx_mul, scap * 4) != hipSuccess ||
            pool_malloc(t->ctx, &t->lx_w0, cap * 4) != hipSuccess)
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(word lexicon) failed");
        t->lx_cap = scap;
    }
    return sp_grow(t, &t->lx_occ, &t->lx_occ_cap, ocap);
}

// zone buffers (zeroed): the zone, and the stale source (previous stream,
// n_prev - Zs <= z + prev_mc symbols), at least the one-workgroup zone pass's full
// register window, which it loads unconditionally
int sp_alloc_zone(gbpe_trainer* t, uint64_t z, uint64_t prev_mc) {
    hipStream_t s = t->ctx->stream;
    uint64_t zneed = (gbpe_div_up(z + prev_mc + 1, TILE) + 2) * TILE;
    const uint64_t zmin = (uint64_t)(t->u16 ? zone_max<uint16_t>(1024) : zone_max<uint32_t>(1024)) + TILE;
    if (zneed < zmin) zneed = zmin;
    if (zneed > t->zcap) {
        for (int k = 0; k < 2; ++k) {
            pool_free(t->ctx, t->zbuf[k]);
            t->zbuf[k] = nullptr;
        }
        pool_free(t->ctx, t->wtmp);
        t->wtmp = nullptr;
        t->zcap = 0;
        if (pool_malloc(t->ctx, &t->zbuf[0], zneed * t->bps) != hipSuccess || pool_malloc(t->ctx, &t->zbuf[1], zneed * t->bps) != hipSuccess ||
            pool_malloc(t->ctx, &t->wtmp, zneed * t->bps) != hipSuccess)
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(zone) failed");
        t->zcap = zneed;
    }
    {   // delta dumps of the multi-tile zone passes: the most tile workgroups a pass can have
        const uint64_t zt = gbpe_div_up(t->zcap, TILE);
        const uint32_t need = (uint32_t)std::max<uint64_t>(std::min<uint64_t>(zt, t->delta_mt ? t->delta_mt : zt),
                                                           gbpe_div_up(zt, 8)) + 1;
        if (t->zdr_on && need > t->zdr_ntile) {
            pool_free(t->ctx, t->zdr_out);
            pool_free(t->ctx, t->zdr_offs);
            pool_free(t->ctx, t->zdr_flag);
            t->zdr_out = nullptr, t->zdr_offs = nullptr, t->zdr_flag = nullptr;
            t->zdr_ntile = 0;
            const uint64_t nd = (uint64_t)need + ZDR_P;
            if (pool_malloc(t->ctx, &t->zdr_out, ((uint64_t)need * ZDR_N_TILE + (uint64_t)ZDR_P * ZDR_N_CHURN) * sizeof(uint2)) !=
                    hipSuccess ||
                pool_malloc(t->ctx, &t->zdr_offs, nd * (ZDR_P + 1) * 4) != hipSuccess || pool_malloc(t->ctx, &t->zdr_flag, nd * 4) != hipSuccess)
                return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(zone delta dumps) failed");
            TR_HIP(t, hipMemsetAsync(t->zdr_flag, 0, nd * 4, s));   // tags start at 1
            t->zdr_ntile = need;
        }
    }
    for (int k = 0; k < 2; ++k) TR_HIP(t, hipMemsetAsync(t->zbuf[k], 0, t->zcap * t->bps, s));
    return GBPE_OK;
}

// the states of a sparse entry: zone state (length z), body length Zs in the
// global state, the zone rule's fields; per-k_body-workgroup byte counters, the
// k_refresh partial maxima, the zone-segment hand-off.  The caller then runs a
// k_refresh (block maxima + partial maxima) before the first sparse merge.
int sp_init_states(gbpe_trainer* t, uint64_t cap, uint32_t Zs, uint32_t z, uint32_t zlast) {
    hipStream_t s = t->ctx->stream;
    if (!t->zst) {
        TR_HIP(t, pool_malloc(t->ctx, &t->zst, sizeof(DevState)));
        TR_HIP(t, pool_hmalloc(t->ctx, &t->h_zst, sizeof(DevState)));
    }
    memset(t->h_zst, 0, sizeof(DevState));
    t->h_zst->n = z;
    TR_HIP(t, hipMemcpyAsync(t->zst, t->h_zst, sizeof(DevState), hipMemcpyHostToDevice, s));
    t->h_st->B = Zs;
    t->h_st->Bp = Zs;
    t->h_st->body_rm = 0;
    t->h_st->sp_abort = 0;
    TR_HIP(t, hipMemcpyAsync(&t->st->B, &t->h_st->B, 4 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    // every rank checks the zone against the same length: the zone rank's target
    // until the first exchange reports the real one (single GPU: the real one)
    t->h_st->zlast = zlast;
    t->h_st->is_last = z ? 1u : 0u;
    TR_HIP(t, hipMemcpyAsync(&t->st->zlast, &t->h_st->zlast, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->st->is_last, &t->h_st->is_last, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    {   // one byte counter per k_body workgroup, kept across entries (summed by gbpe_trainer_stats_get)
        const uint64_t need = std::max<uint64_t>(gbpe_div_up(gbpe_div_up(cap, 32), SP_WPW_MIN), t->body_cap) + 2;
        if (need > t->wg_cap) {
            uint64_t* nb = nullptr;
            TR_HIP(t, pool_malloc(t->ctx, &nb, need * sizeof(uint64_t)));
            TR_HIP(t, hipMemsetAsync(nb, 0, need * sizeof(uint64_t), s));
            if (t->wg_bytes) TR_HIP(t, hipMemcpyAsync(nb, t->wg_bytes, t->wg_cap * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
            TR_HIP(t, hipStreamSynchronize(s));
            pool_free(t->ctx, t->wg_bytes);
            t->wg_bytes = nb;
            t->wg_cap = need;
        }
    }
    // the zone rule's last count (sel_inline): the count of the merge before entry
    TR_HIP(t, hipMemcpyAsync(&t->st->mc_prev, &t->st->mc, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    // per-k_refresh-workgroup maxima the sparse merges select from (sel_inline)
    if (!t->part) {
        int rc = part_alloc(t);
        if (rc != GBPE_OK) return rc;
    }
    if (!t->zseg) {
        TR_HIP(t, pool_malloc(t->ctx, &t->zseg, sizeof(ZSegState)));
        TR_HIP(t, hipMemsetAsync(t->zseg, 0, sizeof(ZSegState), t->ctx->stream));
    }
    if (!t->d_u32) TR_HIP(t, pool_malloc(t->ctx, &t->d_u32, 64));
    return GBPE_OK;
}

// dense → sparse at a step boundary.  The zone is the stream from the last word
// start at or before n - zt (zt = max(sp_zt * next_mc, 2 next_mc + last_mc) + 64:
// >= 5 x the next merge's count while counts fall, and room for the stale window
// the last merge left (sel_inline's zone rule); a merge that would not fit is not
// run and the host goes dense, sp_abort); the dense stale buffer's tail becomes the
// zone's stale buffer.  next_mc = 0: the last merge's count stands in for it.
template <typename S>
int sp_enter(gbpe_trainer* t, bool with_zone = true, uint32_t next_mc = 0) {
    hipStream_t s = t->ctx->stream;
    const uint32_t n = (uint32_t)t->n;
    const uint64_t prev_mc = t->last_mc;   // the previous stream is n + prev_mc long
    const uint64_t nmc = next_mc ? next_mc : prev_mc;
    const uint64_t zt = std::max<uint64_t>((uint64_t)t->sp_zt * nmc, 2ull * nmc + prev_mc) + 64;
    const S* cur = (const S*)t->buf[t->cur];
    const S* stale = (const S*)t->buf[t->cur ^ 1];
    if (!t->d_u32) TR_HIP(t, pool_malloc(t->ctx, &t->d_u32, 64));
    uint32_t Zs = n;
    if (with_zone) {
        if (zt + 2 >= n) return GBPE_OK;
        hipLaunchKernelGGL(k_sp_zone_start<S>, dim3(1), dim3(1024), 0, s, cur, (uint32_t)(n - zt), t->d_u32);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipMemcpyAsync(&Zs, t->d_u32, 4, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
        if (Zs < t->sp_secw) return GBPE_OK;   // the whole stream is one long word (or tiny): stay dense
    }
    const uint32_t z = n - Zs;
    // word lexicon: plan the deduplicated body first; it sizes the sectors
    t->lex = false;
    t->lx_len = t->lx_nocc = 0;
    t->lx_nuid = 0;
    LxPlan lp;
    if (t->lex_on && Zs) {
        int rc0 = lx_analyze<S>(t, cur, Zs, true, lp);
        if (rc0 != GBPE_OK) return rc0;
        if (lp.ok) ++t->lx_builds;
        else ++t->lx_fallbacks;
    }
    // sector capacity: windows over [0, n) (the lexicon: over its store, with room
    // for a 16th of the zone's symbols as the words shrinks append; sp_reserve grows
    // it) plus one partial window per zone shrink (at most SP_SHRINKS per entry)
    const uint64_t cap = lp.ok ? gbpe_div_up((uint64_t)lp.T + z / 16, t->sp_secw) + 2 * (SP_SHRINKS + 1)
                               : gbpe_div_up(n, t->sp_secw) + SP_SHRINKS + 1;
    int rc = sp_alloc_layout(t, cap);
    if (rc != GBPE_OK) return rc;
    t->bcur = t->cur;
    if (lp.ok) {
        rc = sp_alloc_lexicon(t, cap, (uint64_t)lp.nw + z / 16 + 1024);
        if (rc != GBPE_OK) return rc;
        t->lex = true;
        rc = lx_commit<S>(t, lp, cur, true);
        if (rc == GBPE_OK && !lp.ok) rc = gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "word lexicon capacity");
        if (rc == GBPE_OK && gbpe_debug_knob("lex_check", 0)) rc = lx_check<S>(t, cur, Zs, lp);
    } else {
        rc = sp_add_sectors<S>(t, 0u, Zs);
    }
    if (rc != GBPE_OK) return rc;
    t->sp_age = 0;
    t->sp_bits_age = 0;
    t->sp_shrinks = 0;
    rc = sp_alloc_zone(t, z, prev_mc);
    if (rc != GBPE_OK) return rc;
    if (z) {
        TR_HIP(t, hipMemcpyAsync(t->zbuf[0], cur + Zs, (uint64_t)z * t->bps, hipMemcpyDeviceToDevice, s));
        uint64_t sl = (uint64_t)z + prev_mc;
        if (Zs + sl > t->cap_syms) sl = t->cap_syms - Zs;
        if (sl > t->zcap) sl = t->zcap;
        TR_HIP(t, hipMemcpyAsync(t->zbuf[1], stale + Zs, sl * t->bps, hipMemcpyDeviceToDevice, s));
    }
    rc = sp_init_states(t, cap, Zs, z, z);
    if (rc != GBPE_OK) return rc;
    GBPE_LAUNCH_REFRESH(S, t->g_refresh, t->tb.nblk, s, t->st, 0u, 0, t->tb, (S*)nullptr, (const uint32_t*)nullptr,
                        (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(), t->part, (uint32_t*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    TR_HIP(t, hipStreamSynchronize(s));
    t->sp = true;
    t->zcur = 0;
    if (t->last_mc < nmc) t->last_mc = (uint32_t)nmc;   // the zone-shrink target's count until a merge runs
    ++t->sp_enters;
    t->sp_sectors = t->nsec;
    t->sp_zone = z;
    return GBPE_OK;
}

// Zone shrink at a step boundary: the zone keeps >= zt = sp_zt * last_mc + 64
// symbols (from a word start); its front moves into the body as new sectors and
// both zone buffers shift down by the moved length (B and Bp with them, so the
// stale buffer keeps its global coordinates).
template <typename S>
int sp_shrink(gbpe_trainer* t) {
    hipStream_t s = t->ctx->stream;
    DevState* hs = t->h_st;
    const uint32_t z = (uint32_t)t->n - hs->B;
    const uint64_t zt = (uint64_t)t->sp_zt * t->last_mc + 64;
    // paired launches run in the zone_one form: a zone just above it whose target fits
    // shrinks into it (else it stays there until z >= 2 zt + 4096: 1 GiB merges ~12K-25K)
    const uint64_t zmax1 = zone_max<S>(256);
    const bool to_one = t->pair_on && t->pair_one && z > zmax1 && zt + 512 <= zmax1;
    if (t->sp_shrinks >= SP_SHRINKS_MAX || ((uint64_t)z < zt * t->shrink_pct / 100 + 4096 && !to_one)) return GBPE_OK;
    S* zc = (S*)t->zbuf[t->zcur];
    S* zo = (S*)t->zbuf[t->zcur ^ 1];
    hipLaunchKernelGGL(k_sp_zone_start<S>, dim3(1), dim3(1024), 0, s, (const S*)zc, (uint32_t)(z - zt), t->d_u32);
    GBPE_LAUNCH_CHECK(t->ctx);
    uint32_t L = 0;
    TR_HIP(t, hipMemcpyAsync(&L, t->d_u32, 4, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (L < (to_one ? 512u : 4096u)) return GBPE_OK;
    if (t->lex) {   // the front's words join the lexicon (deduplicated among themselves)
        LxPlan lp;
        int rc = lx_analyze<S>(t, (const S*)zc, L, false, lp);
        if (rc == GBPE_OK && lp.ok) rc = lx_commit<S>(t, lp, (const S*)zc, false);
        if (rc != GBPE_OK) return rc;
        if (!lp.ok) return GBPE_OK;   // (a collision or no room): the zone keeps its front this time
    } else {
        if ((uint64_t)t->bend + L > t->cap_syms) return GBPE_OK;
        S* body = (S*)t->buf[t->bcur];
        TR_HIP(t, hipMemcpyAsync(body + t->bend, zc, (uint64_t)L * t->bps, hipMemcpyDeviceToDevice, s));
        int rc = sp_add_sectors<S>(t, t->bend, L);
        if (rc != GBPE_OK) return rc;
    }
    // both buffers shift down by L.  Only their live extents move: the zone [0, z)
    // and the stale buffer, which the next window reads below the previous zone
    // length (<= z + last_mc); the buffers' capacity is the zone at entry (~200M
    // symbols at 1 GiB), so moving all of it cost ~1 ms per late shrink.
    const uint64_t live = std::min<uint64_t>(t->zcap, (uint64_t)z + 2ull * t->last_mc + 2ull * TILE);
    const uint64_t rest = live - L;
    TR_HIP(t, hipMemcpyAsync(t->wtmp, zc + L, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemcpyAsync(zc, t->wtmp, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemcpyAsync(t->wtmp, zo + L, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemcpyAsync(zo, t->wtmp, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemsetAsync(zc + rest, 0, (uint64_t)L * t->bps, s));
    TR_HIP(t, hipMemsetAsync(zo + rest, 0, (uint64_t)L * t->bps, s));
    hs->B += L;
    hs->Bp += L;
    t->h_zst->n = z - L;
    TR_HIP(t, hipMemcpyAsync(&t->st->B, &hs->B, 2 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->zst->n, &t->h_zst->n, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    ++t->sp_shrinks;
    return GBPE_OK;
}

// sparse → dense: the body sectors gathered in order into the other dense
// buffer, the zone appended; the old body buffer becomes the stale buffer, with
// the zone's stale buffer at its global place (positions >= Bp: the only ones the
// next merge's stale window can read).
template <typename S>
int sp_exit(gbpe_trainer* t) {
    if (t->lex_only)
        return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "a trainer built from shard lexicons cannot return to one dense "
                              "stream (a merge outgrew the zone, or the stream was asked for: use gbpe_trainer_expand)");
    hipStream_t s = t->ctx->stream;
    DevState* hs = t->h_st;
    TR_HIP(t, hipMemcpyAsync(hs, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    const uint32_t B = hs->B, Bp = hs->Bp, n = hs->n;
    const uint32_t z = n - B;
    S* body = (S*)t->buf[t->bcur];
    S* dst = (S*)t->buf[t->bcur ^ 1];
    const uint32_t nsec = t->nsec;
    uint64_t btot = 0;
    if (t->lex) {
        int rc = lx_expand<S>(t, dst, (uint64_t)B, &btot);
        if (rc != GBPE_OK) return rc;
    } else {
        hipLaunchKernelGGL(k_sp_counts, dim3((uint32_t)gbpe_div_up(nsec, 256)), dim3(256), 0, s, (const uint2*)t->sec, nsec,
                           t->sp_loc);
        const uint64_t nblk = gbpe_div_up(nsec, SCAN_BLK);
        hipLaunchKernelGGL(k_chunk_scan1, dim3((uint32_t)nblk), dim3(SCAN_TPB), 0, s, (const uint32_t*)t->sp_loc,
                           (uint64_t)nsec, t->sp_loc, t->sp_blk);
        hipLaunchKernelGGL(k_chunk_scan2, dim3(1), dim3(SCAN_TPB), 0, s, t->sp_blk, nblk, t->sp_blk + nblk);
        hipLaunchKernelGGL(k_sp_gather<S>, dim3((uint32_t)gbpe_div_up(nsec, TPB / 64)), dim3(TPB), 0, s, (const S*)body,
                           (const uint2*)t->sec, nsec, (const uint32_t*)t->sp_loc, (const uint64_t*)t->sp_blk, dst);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipMemcpyAsync(&btot, t->sp_blk + nblk, 8, hipMemcpyDeviceToHost, s));
    }
    TR_HIP(t, hipMemcpyAsync(dst + B, t->zbuf[t->zcur], (uint64_t)z * t->bps, hipMemcpyDeviceToDevice, s));
    // zero the rest of the dense buffer's padding the kernels may read (halo / look-ahead)
    TR_HIP(t, hipMemsetAsync(dst + n, 0, (t->cap_syms - n) * t->bps, s));
    uint64_t sl = t->zcap;
    if (Bp + sl > t->cap_syms) sl = t->cap_syms - Bp;
    TR_HIP(t, hipMemcpyAsync(body + Bp, t->zbuf[t->zcur ^ 1], sl * t->bps, hipMemcpyDeviceToDevice, s));
    hs->sp_abort = 0;
    TR_HIP(t, hipMemcpyAsync(&t->st->sp_abort, &hs->sp_abort, 4, hipMemcpyHostToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (btot != B) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "sparse exit: body sectors hold %llu symbols, expected %u",
                                         (unsigned long long)btot, B);
    t->cur = t->bcur ^ 1;
    t->sp = false;
    t->lex = false;
    ++t->sp_exits;
    return GBPE_OK;
}

// options and environment knobs of a new trainer; symbol width from the ids the run can make
void trainer_config(gbpe_trainer* t, gbpe_ctx* ctx, const gbpe_train_opts* opts) {
    t->ctx = ctx;
    t->flags = opts->flags;
    t->batch = opts->batch_size ? opts->batch_size : GBPE_BATCH_SIZE;
    const uint32_t vocab_size = opts->vocab_size ? opts->vocab_size : 256u;
    const uint32_t next_id = opts->next_token_id ? opts->next_token_id : 256u;
    t->next_id0 = next_id;
    t->needed = opts->target_vocab_size > vocab_size ? opts->target_vocab_size - vocab_size : 0u;
    // u16 symbols when every id the run can produce fits in 15 bits
    const uint64_t max_id = (uint64_t)next_id + t->needed;    // exclusive
    t->u16 = max_id <= 0x8000ull;
    t->max_id = (uint32_t)(max_id < 0x10000ull ? max_id : 0x10000ull);
    t->body_cap = (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256);
    t->body_cap = (uint32_t)std::max<long>(1, gbpe_debug_knob("bcap", t->body_cap));
    t->z256 = (uint32_t)gbpe_debug_knob("z256", t->z256);
    t->seg8 = (uint32_t)gbpe_debug_knob("seg8", t->seg8);
    t->zseg_lo = (uint32_t)std::max<long>(8192, gbpe_debug_knob("zslo", t->zseg_lo));   // one per CU: measured best at 1 GiB (128/192/256/384/512/1024: 3.01/2.42/2.14/2.66/2.45/2.98 s)
    // test overrides (GBPE_DEBUG): the lexicon off / its build check, the
    // in-loop table growth off, the multi-tile k_delta threshold, the zone target
    t->lex_on = gbpe_debug_knob("lexicon", 1) != 0;
    t->body_fit = gbpe_debug_knob("bodyfit", 1) != 0;
    t->pair_on = gbpe_debug_knob("pair", 1) != 0;
    t->pair_one = gbpe_debug_knob("pone", 1) != 0;
    t->ptrace = (uint32_t)gbpe_debug_knob("ptrace", 0);
    t->rehash_on = gbpe_debug_knob("rehash", 1) != 0;
    t->delta_mt = (uint32_t)gbpe_debug_knob("delta_mt", t->delta_mt);
    t->sp_zt = (uint32_t)gbpe_debug_knob("zt", t->sp_zt);
    t->grow_used_pct = (uint32_t)std::min<long>(90, std::max<long>(10, gbpe_debug_knob("gused", t->grow_used_pct)));
    t->grow_live_pct = (uint32_t)std::min<long>(t->grow_used_pct, std::max<long>(5, gbpe_debug_knob("glive", t->grow_live_pct)));
    t->refresh_blocks = (uint32_t)gbpe_debug_knob("rfb", t->refresh_blocks);   // k_refresh grid sweeps
    t->refresh_late = (uint32_t)gbpe_debug_knob("rfl", t->refresh_late);
    t->refresh_late_z = (uint32_t)gbpe_debug_knob("rflz", t->refresh_late_z);
    t->lx_div = (uint32_t)std::max<long>(1, gbpe_debug_knob("lxdiv", t->lx_div));   // lexicon entry / sub-step sweeps
    t->lx_wg = (uint32_t)std::max<long>(1, gbpe_debug_knob("lxwg", t->lx_wg));
    t->lx_two = gbpe_debug_knob("lxtwo", 1) != 0;
    t->htime = (uint32_t)gbpe_debug_knob("htime", 0);
    t->body_min = (uint32_t)std::max<long>(1, gbpe_debug_knob("bmin", t->body_min));
    t->body_sub = (uint32_t)std::min<long>(4, std::max<long>(1, gbpe_debug_knob("bsub", t->body_sub)));
    t->sub_k = (uint32_t)std::max<long>(1, gbpe_debug_knob("subk", t->sub_k));
    t->sub_zone = (uint32_t)std::max<long>(1, gbpe_debug_knob("subz", t->sub_zone));
    if (t->sp_zt < t->zone_f) t->sp_zt = t->zone_f;
    if (const char* e = getenv("GBPE_SPARSE_TRACE")) {
        t->trace = fopen(e, "w");
        if (t->trace && (pool_malloc(t->ctx, &t->d_clog, (size_t)t->batch * 8) != hipSuccess ||
                         pool_hmalloc(t->ctx, &t->h_clog, (size_t)t->batch * 8) != hipSuccess))
            t->d_clog = nullptr, t->h_clog = nullptr;   // trace without candidate counts
    }
    t->bps = t->u16 ? 2 : 4;
}

int sp_exit_any(gbpe_trainer* t) { return !t->sp ? GBPE_OK : (t->u16 ? sp_exit<uint16_t>(t) : sp_exit<uint32_t>(t)); }

}  // namespace

// a trainer continuing from an exported state (gbpe_trainer_create_from_state):
// `bytes` is then the current u32 stream, `prev` the previous one
struct StateInit {
    const uint32_t* prev;
    uint64_t n_prev;
};
// the trainer constructor behind gbpe_trainer_create / _create_from_state (and, through
// trainer_config, _create_from_lexicon)
int trainer_create_impl(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                        int input_on_device, const gbpe_train_opts* opts, uint64_t cap_extra, gbpe_trainer** out,
                        const StateInit* si = nullptr);
