// Sharded first pass + lexicon hand-over.
//
// The reference trains one vocabulary on one WebGPU device (training-pipeline.js:
// 178-222): its merge chain is sequential, every merge's argmax needing the counts
// after the previous one.  What does parallelise is the first pass: symbols, word
// boundaries (train.wgsl:87-186), pair counts (train.wgsl:366-431, additive across
// word-start shards: train.wgsl:395, 483, 493) and the word lexicon of DESIGN §2c.
// So every rank runs that pass on its piece of the corpus (a gbpe_lexshard), the
// pieces' distinct words (one store per rank, every word with its multiplicity)
// go to ONE root, which deduplicates them into one global lexicon, takes the dense
// zone (the stream's tail, where the reference compaction quirk of train.wgsl:
// 605-607 + 698/727 acts) from the last rank, counts the pairs from the lexicon and
// the zone, and runs the single-device sector-sparse loop from the first merge.
// The stream never has to sit on one device: the root holds the distinct words
// (C4 at 8 GiB: ~10^8 store symbols for 8.6*10^9 stream symbols) and the zone; the
// stream order of the body stays on the ranks (their occurrence lists, remapped to
// the root's word ids), which is all gbpe_trainer_expand needs to rebuild the
// final stream.  Host protocol: gpu-bpe_amd/gpubpe/lexshard.py.

#include "trainer.h"

struct gbpe_lexshard {
    gbpe_ctx* ctx = nullptr;
    gbpe_trainer* t = nullptr;   // the piece's symbols + pair counts (dense trainer), until release
    bool u16 = true;
    uint32_t bps = 2;
    uint64_t n = 0, Zs = 0, z = 0;
    uint32_t top = 0;            // the piece's largest pair count
    void* store = nullptr;       // distinct words, each followed by a 0 separator (S layout)
    uint32_t* mul = nullptr;     // per store symbol: its word's occurrences in the piece
    uint64_t T = 0;
    uint32_t* occ = nullptr;     // the piece's body words in stream order: local uid (global after remap) or LX_LIT
    uint64_t nw = 0;
    uint32_t nu = 0;
    void* zone = nullptr;        // the piece's zone (last rank): symbols [Zs, n)
    bool built = false, remapped = false;
};

namespace {

// pair counts of a segment into the table, every pair weighted by w[its right
// symbol] (a word store's multiplicities) or 1 (w null) — the counting rule of
// train.wgsl:393-399; pairs never span a 0 separator or a word start
template <typename S>
__global__ __launch_bounds__(TPB) void k_count_seg(const S* __restrict__ x, const uint32_t* __restrict__ w, uint64_t len,
                                                   Table tb, DevState* st) {
    __shared__ LdsTab<LTAB_FULL> lt;
    lds_clear(lt);
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * TPB;
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x + 1; i < len; i += stride) {
        const uint32_t x1 = x[i], x0 = x[i - 1];
        const uint32_t t0 = x0 & Sym<S>::TM, t1 = x1 & Sym<S>::TM;
        if (!(x1 & Sym<S>::WS) && t0 && t1) lds_add(lt, tb, st, (t0 << 16) | t1, w ? w[i] : 1u);
    }
    lds_flush(lt, tb, st);
}

// the concatenated stores are words and separators alternately: entry j is word
// 2j of the analysis, so its global uid is occ[2j]
__global__ void k_lx_map(const uint32_t* __restrict__ occ, uint64_t nent, uint32_t* __restrict__ map,
                         uint32_t* __restrict__ bad) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nent) return;
    const uint32_t o = occ[2 * j], sep = occ[2 * j + 1];
    if ((o & LX_LIT) || !(sep & LX_LIT) || (sep & ~LX_LIT)) *bad = 1u;
    map[j] = o;
}

// a piece's occurrence list to global uids (literals stay)
__global__ void k_lx_remap(uint32_t* __restrict__ occ, uint64_t nw, const uint32_t* __restrict__ map, uint64_t nmap,
                           uint32_t* __restrict__ bad) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nw) return;
    const uint32_t o = occ[j];
    if (o & LX_LIT) return;
    if (o >= nmap) {
        *bad = 1u;
        return;
    }
    occ[j] = map[o];
}

template <typename S>
int ls_build(gbpe_lexshard* ls, uint64_t zone_target) {
    gbpe_trainer* t = ls->t;
    hipStream_t s = ls->ctx->stream;
    const S* cur = (const S*)t->buf[t->cur];
    const uint64_t n = t->n;
    uint32_t Zs = (uint32_t)n;
    if (zone_target >= n) {   // the whole piece lies inside the zone (a zone spanning several pieces)
        Zs = 0;
    } else if (zone_target) {   // the piece's tail from the last word start at or before n - zone_target
        hipLaunchKernelGGL(k_sp_zone_start<S>, dim3(1), dim3(1024), 0, s, cur, (uint32_t)(n - zone_target), t->d_u32);
        GBPE_LAUNCH_CHECK(ls->ctx);
        TR_HIP(t, hipMemcpyAsync(&Zs, t->d_u32, 4, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
    }
    LxPlan lp;
    int rc = lx_analyze<S>(t, cur, Zs, false, lp);
    if (rc != GBPE_OK) return rc;
    if (Zs && !lp.ok)
        return gbpe_set_error(ls->ctx, GBPE_E_INTERNAL, "lexshard: word lexicon build failed (word table full or a "
                                                        "64-bit word-hash collision)");
    ls->Zs = Zs;
    ls->z = n - Zs;
    ls->T = lp.T;
    ls->nu = lp.nu;
    ls->nw = lp.nw;
    const uint64_t T = lp.T;
    if (pool_malloc(ls->ctx, &ls->store, (T + 64) * ls->bps) != hipSuccess ||
        pool_malloc(ls->ctx, &ls->mul, (T + 64) * 4) != hipSuccess || pool_malloc(ls->ctx, &ls->occ, (lp.nw + 1) * 4) != hipSuccess ||
        (ls->z && pool_malloc(ls->ctx, &ls->zone, (ls->z + 64) * ls->bps) != hipSuccess))
        return gbpe_set_error(ls->ctx, GBPE_E_OOM, "lexshard: hipMalloc(store) failed");
    if (lp.nu)
        hipLaunchKernelGGL(k_lx_fill<S>, dim3((uint32_t)gbpe_div_up(lp.nu, 256)), dim3(256), 0, s, cur,
                           (const uint32_t*)lp.urep, (const uint32_t*)lp.usz, (const uint32_t*)lp.umul,
                           (const uint32_t*)lp.upre, (const uint64_t*)lp.ublk, lp.nu, (S*)ls->store, ls->mul);
    GBPE_LAUNCH_CHECK(ls->ctx);
    if (lp.nw) TR_HIP(t, hipMemcpyAsync(ls->occ, lp.occ, lp.nw * 4, hipMemcpyDeviceToDevice, s));
    if (ls->z) TR_HIP(t, hipMemcpyAsync(ls->zone, cur + Zs, ls->z * ls->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    ls->built = true;
    return GBPE_OK;
}

// the hand-over's trainer (gbpe_trainer_create_from_lexicon), from device buffers
// GBPE_DEBUG=rtime=1: the hand-over root's phases to stderr (stream-synchronised wall times)
struct RootTimer {
    bool on;
    hipStream_t s;
    std::chrono::steady_clock::time_point t0;
    RootTimer(hipStream_t s_) : on(gbpe_debug_knob("rtime", 0) != 0), s(s_), t0(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        (void)hipStreamSynchronize(s);
        const auto t1 = std::chrono::steady_clock::now();
        fprintf(stderr, "[gbpe root] %-10s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    }
};

template <typename S>
int lex_root_build(gbpe_trainer* t, const S* store, const uint32_t* mul, uint64_t T, const S* zone, uint64_t z,
                   uint64_t body_len, uint32_t* d_map, uint64_t* n_map, RootTimer& rt) {
    gbpe_ctx* ctx = t->ctx;
    hipStream_t s = ctx->stream;
    // weighted analysis of the concatenated stores: one global uid per distinct word
    LxPlan lp;
    int rc = lx_analyze<S>(t, store, (uint32_t)T, false, lp, mul);
    if (rc != GBPE_OK) return rc;
    rt.mark("analyze");
    if (T && !lp.ok)
        return gbpe_set_error(ctx, GBPE_E_INTERNAL, "lexicon hand-over: global word table full or a 64-bit word-hash "
                                                    "collision");
    if (lp.nw & 1u) return gbpe_set_error(ctx, GBPE_E_INVALID, "lexicon hand-over: the stores are not word/separator pairs");
    const uint64_t nent = lp.nw / 2;
    *n_map = nent;
    if (nent) {
        hipLaunchKernelGGL(k_lx_map, dim3((uint32_t)gbpe_div_up(nent, 256)), dim3(256), 0, s, (const uint32_t*)lp.occ,
                           nent, d_map, t->d_u32 + 1);
        GBPE_LAUNCH_CHECK(ctx);
    }
    // sectors, bitmap, signatures, store (the body is the deduplicated store)
    const uint64_t cap = gbpe_div_up((uint64_t)lp.T + z / 16, t->sp_secw) + 2 * (SP_SHRINKS + 1);   // (sp_reserve grows it)
    rc = sp_alloc_layout(t, cap);
    if (rc == GBPE_OK) rc = sp_alloc_lexicon(t, cap, z / 16 + 1024);   // occurrences: the zone fronts shrinks move in
    if (rc != GBPE_OK) return rc;
    t->lex = true;
    t->lx_len = t->lx_nocc = 0;
    t->lx_nuid = 0;
    rc = lx_commit<S>(t, lp, store, true, false);
    if (rc == GBPE_OK && !lp.ok) rc = gbpe_set_error(ctx, GBPE_E_INTERNAL, "lexicon hand-over: store capacity");
    if (rc != GBPE_OK) return rc;
    ++t->lx_builds;
    rt.mark("commit");
    // the zone; its stale source is all 0 (no merge has run: both ping-pong buffers
    // start zeroed, as WebGPU zero-initialises buffers)
    rc = sp_alloc_zone(t, z, 0);
    if (rc != GBPE_OK) return rc;
    if (z) TR_HIP(t, hipMemcpyAsync(t->zbuf[0], zone, z * t->bps, hipMemcpyDeviceToDevice, s));
    // the zone passes' tile scratch
    const uint64_t ntz = gbpe_div_up(t->zcap, TILE) + 1;
    if (pool_malloc(t->ctx, &t->hitmask, ntz * TPB * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tile_cnt, ntz * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->grpsum, (ntz / GRP + 2) * GSTR * sizeof(uint32_t)) != hipSuccess)
        return gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(zone scratch) failed");
    TR_HIP(t, hipMemsetAsync(t->hitmask, 0, ntz * TPB * sizeof(uint32_t), s));
    // pair counts: the store weighted by its multiplicities, plus the zone
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    TR_HIP(t, hipMemsetAsync(t->tb.slots, 0, slots * sizeof(uint2), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax2, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.blive, 0, (uint64_t)t->tb.nblk * sizeof(uint32_t), s));
    TR_HIP(t, hipMemsetAsync(&t->st->used, 0, sizeof(uint32_t), s));
    if (t->lx_len > 1)
        hipLaunchKernelGGL(k_count_seg<S>, dim3(grid_persistent(ctx, gbpe_div_up(t->lx_len, TILE), 2)), dim3(TPB), 0, s,
                           (const S*)t->lx_store, (const uint32_t*)t->lx_mul, t->lx_len, t->tb, t->st);
    if (z > 1)
        hipLaunchKernelGGL(k_count_seg<S>, dim3(grid_persistent(ctx, gbpe_div_up(z, TILE), 2)), dim3(TPB), 0, s,
                           (const S*)t->zbuf[0], (const uint32_t*)nullptr, z, t->tb, t->st);
    hipLaunchKernelGGL(k_clear_dirty_all, dim3(gbpe_div_up(t->tb.nblk, 256)), dim3(256), 0, s, t->st, t->tb);
    hipLaunchKernelGGL(k_refresh<S>, dim3(grid_blocks(ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st, 0u, 0, t->tb,
                       (S*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    hipLaunchKernelGGL(k_topcount, dim3(1), dim3(1024), 0, s, t->tb, t->d_u32);
    GBPE_LAUNCH_CHECK(ctx);
    rt.mark("zone+count");
    uint32_t hs[2] = {0, 0};
    TR_HIP(t, hipMemcpyAsync(hs, t->d_u32, 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (hs[1]) return gbpe_set_error(ctx, GBPE_E_INVALID, "lexicon hand-over: the stores are not word/separator pairs");
    t->last_mc = hs[0];   // the zone-shrink target's count until a merge runs (as sp_enter)
    // states: body = every symbol before the zone (kept modulo 2^32 on the device)
    rc = sp_init_states(t, cap, (uint32_t)body_len, (uint32_t)z, (uint32_t)z);
    if (rc != GBPE_OK) return rc;
    GBPE_LAUNCH_REFRESH(S, t->g_refresh, t->tb.nblk, s, t->st, 0u, 0, t->tb, (S*)nullptr, (const uint32_t*)nullptr,
                        (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(), t->part, (uint32_t*)nullptr);
    GBPE_LAUNCH_CHECK(ctx);
    TR_HIP(t, hipStreamSynchronize(s));
    rt.mark("states");
    t->sp = true;
    t->zcur = 0;
    t->sp_age = t->sp_bits_age = 0;
    t->sp_shrinks = 0;
    ++t->sp_enters;
    t->sp_sectors = t->nsec;
    t->sp_zone = z;
    return GBPE_OK;
}

}  // namespace

// ── rank side ──────────────────────────────────────────────────────────────────

extern "C" int gbpe_lexshard_create(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                                    int input_on_device, const gbpe_train_opts* opts, gbpe_lexshard** out) {
    if (!ctx || !out || !opts) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *out = nullptr;
    auto* ls = new (std::nothrow) gbpe_lexshard();
    if (!ls) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    ls->ctx = ctx;
    // symbols, word boundaries and pair counts of the piece: a dense trainer's creation
    gbpe_train_opts o = *opts;
    o.flags |= GBPE_TRAIN_DENSE_ONLY;
    int rc = trainer_create_impl(ctx, bytes, n, word_starts, input_on_device, &o, 0, &ls->t);
    if (rc != GBPE_OK) {
        delete ls;
        return rc;
    }
    gbpe_trainer* t = ls->t;
    hipStream_t s = ctx->stream;
    // the piece never merges: drop the other ping-pong buffer and the stream-pass scratch
    pool_free(t->ctx, t->buf[t->cur ^ 1]);
    t->buf[t->cur ^ 1] = nullptr;
    pool_free(t->ctx, t->hitmask);
    t->hitmask = nullptr;
    ls->u16 = t->u16;
    ls->bps = t->bps;
    ls->n = t->n;
    if (!t->d_u32 && pool_malloc(t->ctx, &t->d_u32, 64) != hipSuccess) {
        gbpe_lexshard_destroy(ls);
        return gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc failed");
    }
    hipLaunchKernelGGL(k_topcount, dim3(1), dim3(1024), 0, s, t->tb, t->d_u32);
    if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&ls->top, t->d_u32, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        gbpe_lexshard_destroy(ls);
        return gbpe_set_error(ctx, GBPE_E_DEVICE, "lexshard: top count failed");
    }
    *out = ls;
    return GBPE_OK;
}

extern "C" int gbpe_lexshard_build(gbpe_lexshard* ls, uint64_t zone_target) {
    if (!ls || !ls->t) return GBPE_E_INVALID;
    if (ls->built) return gbpe_set_error(ls->ctx, GBPE_E_INVALID, "lexshard: already built");
    return ls->u16 ? ls_build<uint16_t>(ls, zone_target) : ls_build<uint32_t>(ls, zone_target);
}

extern "C" int gbpe_lexshard_info_get(const gbpe_lexshard* ls, gbpe_lexshard_info* o) {
    if (!ls || !o) return GBPE_E_INVALID;
    memset(o, 0, sizeof(*o));
    o->symbols = ls->n;
    o->body = ls->built ? ls->Zs : ls->n;
    o->zone = ls->z;
    o->store_symbols = ls->T;
    o->entries = ls->nu;
    o->words = ls->nw;
    o->top_count = ls->top;
    o->bytes_per_symbol = ls->bps;
    return GBPE_OK;
}

extern "C" int gbpe_lexshard_copy(gbpe_lexshard* ls, int what, void* dst, uint64_t cap_bytes, int dst_on_device) {
    if (!ls || !dst) return GBPE_E_INVALID;
    if (!ls->built) return gbpe_set_error(ls->ctx, GBPE_E_INVALID, "lexshard: not built");
    const void* src = nullptr;
    uint64_t bytes = 0;
    switch (what) {
        case GBPE_LEXSHARD_STORE: src = ls->store, bytes = ls->T * ls->bps; break;
        case GBPE_LEXSHARD_MUL: src = ls->mul, bytes = ls->T * 4; break;
        case GBPE_LEXSHARD_OCC: src = ls->occ, bytes = ls->nw * 4; break;
        case GBPE_LEXSHARD_ZONE: src = ls->zone, bytes = ls->z * ls->bps; break;
        default: return gbpe_set_error(ls->ctx, GBPE_E_INVALID, "lexshard_copy: unknown part %d", what);
    }
    if (bytes > cap_bytes) return gbpe_set_error(ls->ctx, GBPE_E_CAPACITY, "lexshard_copy: need %llu bytes",
                                                 (unsigned long long)bytes);
    if (!bytes) return GBPE_OK;
    hipStream_t s = ls->ctx->stream;
    GBPE_HIP(ls->ctx, hipMemcpyAsync(dst, src, bytes, dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
    GBPE_HIP(ls->ctx, hipStreamSynchronize(s));
    return GBPE_OK;
}

extern "C" int gbpe_lexshard_release(gbpe_lexshard* ls) {
    if (!ls) return GBPE_E_INVALID;
    if (ls->t) {
        gbpe_trainer_destroy(ls->t);
        ls->t = nullptr;
    }
    return GBPE_OK;
}

extern "C" int gbpe_lexshard_remap(gbpe_lexshard* ls, const uint32_t* map, uint64_t n_map, int map_on_device) {
    if (!ls || (!map && n_map)) return GBPE_E_INVALID;
    if (!ls->built || ls->remapped) return gbpe_set_error(ls->ctx, GBPE_E_INVALID, "lexshard_remap: not built or done");
    hipStream_t s = ls->ctx->stream;
    uint32_t* d = nullptr;
    GBPE_HIP(ls->ctx, pool_malloc(ls->ctx, &d, (n_map + 1) * 4 + 8));
    hipError_t e = hipMemsetAsync(d, 0, 4, s);
    if (e == hipSuccess && n_map)
        e = hipMemcpyAsync(d + 1, map, n_map * 4, map_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s);
    if (e == hipSuccess && ls->nw) {
        hipLaunchKernelGGL(k_lx_remap, dim3((uint32_t)gbpe_div_up(ls->nw, 256)), dim3(256), 0, s, ls->occ, ls->nw,
                           (const uint32_t*)(d + 1), n_map, d);
        e = hipGetLastError();
    }
    uint32_t bad = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, d, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    pool_free(ls->ctx, d);
    if (e != hipSuccess) return gbpe_set_error(ls->ctx, GBPE_E_DEVICE, "lexshard_remap: %s", hipGetErrorString(e));
    if (bad) return gbpe_set_error(ls->ctx, GBPE_E_INVALID, "lexshard_remap: a word id outside the map");
    ls->remapped = true;
    return GBPE_OK;
}

extern "C" void gbpe_lexshard_destroy(gbpe_lexshard* ls) {
    if (!ls) return;
    if (ls->ctx && ls->ctx->stream) hipStreamSynchronize(ls->ctx->stream);
    if (ls->t) gbpe_trainer_destroy(ls->t);
    pool_free(ls->ctx, ls->store);
    pool_free(ls->ctx, ls->mul);
    pool_free(ls->ctx, ls->occ);
    pool_free(ls->ctx, ls->zone);
    delete ls;
}

// ── root side ──────────────────────────────────────────────────────────────────

extern "C" int gbpe_trainer_create_from_lexicon(gbpe_ctx* ctx, const void* store, const uint32_t* mul,
                                                uint64_t store_len, const void* zone, uint64_t zone_len,
                                                uint64_t body_len, int input_on_device, const gbpe_train_opts* opts,
                                                uint32_t* map_out, uint64_t map_cap, uint64_t* n_map, int map_on_device,
                                                gbpe_trainer** out) {
    if (!ctx || !out || !opts || !n_map || (store_len && (!store || !mul)) || (zone_len && !zone))
        return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *out = nullptr;
    *n_map = 0;
    if (body_len + zone_len == 0) return gbpe_set_error(ctx, GBPE_E_EMPTY, "No symbols to train on — corpus is empty after pre-processing");
    if (store_len + 2 * TILE >= 0xFFFFFFF0ull)
        return gbpe_set_error(ctx, GBPE_E_INVALID, "lexicon hand-over: %llu store symbols (more than 32 bits)",
                              (unsigned long long)store_len);
    if (zone_len >= (1ull << 31))   // the device keeps n - Bp, a zone-sized length, in 32 bits
        return gbpe_set_error(ctx, GBPE_E_INVALID, "lexicon hand-over: zone of %llu symbols (at most 2^31)",
                              (unsigned long long)zone_len);
    if (zone_len == 0) return gbpe_set_error(ctx, GBPE_E_INVALID, "lexicon hand-over: the stream's tail must be a zone");
    auto* t = new (std::nothrow) gbpe_trainer();
    if (!t) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    trainer_config(t, ctx, opts);
    t->lex_only = true;
    t->n0 = t->n = body_len + zone_len;
    hipStream_t s = ctx->stream;
    RootTimer rt(s);
    auto fail = [&](int code) {
        gbpe_trainer_destroy(t);
        return code;
    };
    // pair table (grown in place when crowded, as in the sector-sparse loop)
    uint32_t lg = opts->table_log2 ? opts->table_log2 : 20;
    if (lg < BLK_LOG2 + 1) lg = BLK_LOG2 + 1;
    if (lg > 28) lg = 28;
    int rc = table_resize(t, lg);
    if (rc != GBPE_OK) return fail(rc);
    if (pool_malloc(t->ctx, &t->st, sizeof(DevState)) != hipSuccess ||
        pool_malloc(t->ctx, &t->d_log, (size_t)t->batch * 4 * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->d_u32, 64) != hipSuccess ||
        pool_hmalloc(t->ctx, &t->h_st, sizeof(DevState)) != hipSuccess ||
        pool_hmalloc(t->ctx, &t->h_log, (size_t)t->batch * 4 * sizeof(uint32_t)) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(training state) failed"));
    t->tb.used = &t->st->used;
    TR_HIP(t, hipMemsetAsync(t->d_u32, 0, 64, s));
    DevState init{};
    init.n = (uint32_t)t->n;
    init.next_id = t->next_id0;
    memcpy(t->h_st, &init, sizeof(init));
    TR_HIP(t, hipMemcpyAsync(t->st, t->h_st, sizeof(DevState), hipMemcpyHostToDevice, s));
    // inputs (and the map) on the device
    const uint64_t bps = t->bps;
    const void* d_store = store;
    const uint32_t* d_mul = mul;
    const void* d_zone = zone;
    void* tmp = nullptr;
    if (!input_on_device) {
        if (pool_malloc(t->ctx, &tmp, store_len * (bps + 4) + zone_len * bps + 64) != hipSuccess)
            return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(hand-over input) failed"));
        char* p = (char*)tmp;
        if ((store_len && (hipMemcpyAsync(p, store, store_len * bps, hipMemcpyHostToDevice, s) != hipSuccess ||
                           hipMemcpyAsync(p + store_len * bps, mul, store_len * 4, hipMemcpyHostToDevice, s) != hipSuccess)) ||
            hipMemcpyAsync(p + store_len * (bps + 4), zone, zone_len * bps, hipMemcpyHostToDevice, s) != hipSuccess) {
            pool_free(t->ctx, tmp);
            return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "hand-over upload failed"));
        }
        d_store = p;
        d_mul = (const uint32_t*)(p + store_len * bps);
        d_zone = p + store_len * (bps + 4);
    }
    rt.mark("upload");
    uint32_t* d_map = nullptr;
    if (pool_malloc(t->ctx, &d_map, (store_len / 2 + 2) * 4) != hipSuccess) {
        pool_free(t->ctx, tmp);
        return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(map) failed"));
    }
    uint64_t nm = 0;
    rc = t->u16 ? lex_root_build<uint16_t>(t, (const uint16_t*)d_store, d_mul, store_len, (const uint16_t*)d_zone,
                                           zone_len, body_len, d_map, &nm, rt)
                : lex_root_build<uint32_t>(t, (const uint32_t*)d_store, d_mul, store_len, (const uint32_t*)d_zone,
                                           zone_len, body_len, d_map, &nm, rt);
    if (rc == GBPE_OK && map_out) {
        if (map_cap < nm) rc = gbpe_set_error(ctx, GBPE_E_CAPACITY, "lexicon hand-over: map needs %llu entries",
                                              (unsigned long long)nm);
        else if (nm && (hipMemcpyAsync(map_out, d_map, nm * 4, map_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                       s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess))
            rc = gbpe_set_error(ctx, GBPE_E_DEVICE, "lexicon hand-over: map copy failed");
    }
    hipStreamSynchronize(s);
    rt.mark("map");
    pool_free(t->ctx, d_map);
    pool_free(t->ctx, tmp);
    *n_map = nm;
    if (rc != GBPE_OK) return fail(rc);
    *out = t;
    return GBPE_OK;
}

namespace {
template <typename S>
int trainer_expand(gbpe_trainer* t, const uint32_t* d_prefix, uint64_t n_prefix, uint32_t* d_out, uint64_t* total) {
    hipStream_t s = t->ctx->stream;
    const uint64_t nown = t->lx_nocc, no = n_prefix + nown;
    uint32_t* occ = nullptr;
    S* tmp = nullptr;
    auto release = gbpe_scope_exit([&] {   // every return path, TR_HIP's included
        pool_free(t->ctx, tmp);
        pool_free(t->ctx, occ);
    });
    const uint64_t z = (uint32_t)t->n - t->h_st->B;
    TR_HIP(t, pool_malloc(t->ctx, &occ, (no + 1) * 4));
    if (n_prefix) TR_HIP(t, hipMemcpyAsync(occ, d_prefix, n_prefix * 4, hipMemcpyDeviceToDevice, s));
    if (nown) TR_HIP(t, hipMemcpyAsync(occ + n_prefix, t->lx_occ, nown * 4, hipMemcpyDeviceToDevice, s));
    // the body's total, then the zone after it
    uint64_t tot = 0;
    if (pool_malloc(t->ctx, &tmp, (t->n + 64) * sizeof(S)) != hipSuccess) {
        tmp = nullptr;
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "expand: hipMalloc(%llu symbols) failed", (unsigned long long)t->n);
    }
    int rc = lx_expand<S>(t, tmp, t->n - z, &tot, occ, no);   // (checks the total before writing)
    TR_HIP(t, hipStreamSynchronize(s));
    if (rc == GBPE_OK && tot + z != t->n)
        rc = gbpe_set_error(t->ctx, GBPE_E_INVALID, "expand: the occurrence lists hold %llu body symbols, the trainer %llu",
                            (unsigned long long)tot, (unsigned long long)(t->n - z));
    if (rc == GBPE_OK) {
        TR_HIP(t, hipMemcpyAsync(tmp + tot, t->zbuf[t->zcur], z * sizeof(S), hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_export_symbols<S>, dim3((uint32_t)gbpe_div_up(t->n, 256)), dim3(256), 0, s, (const S*)tmp,
                           d_out, t->n);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipStreamSynchronize(s));
    }
    *total = tot + z;
    return rc;
}
}  // namespace

extern "C" int gbpe_trainer_expand(gbpe_trainer* t, const uint32_t* prefix_occ, uint64_t n_prefix, int prefix_on_device,
                                   uint32_t* out, uint64_t cap, uint64_t* n_out, int out_on_device) {
    if (!t || !n_out || (n_prefix && !prefix_occ)) return GBPE_E_INVALID;
    *n_out = t->n;
    if (!out) return GBPE_OK;
    if (!t->sp || !t->lex) return gbpe_set_error(t->ctx, GBPE_E_INVALID, "expand: the trainer holds no word lexicon");
    if (cap < t->n) return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "expand: need %llu", (unsigned long long)t->n);
    hipStream_t s = t->ctx->stream;
    TR_HIP(t, hipMemcpyAsync(t->h_st, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    uint32_t* d_pre = nullptr;
    uint32_t* d_out = out_on_device ? out : nullptr;
    uint32_t* d_own = nullptr;   // the staging output this call allocated
    auto release = gbpe_scope_exit([&] {   // every return path, TR_HIP's included
        pool_free(t->ctx, d_pre);
        pool_free(t->ctx, d_own);
    });
    if (n_prefix && !prefix_on_device) {
        TR_HIP(t, pool_malloc(t->ctx, &d_pre, n_prefix * 4));
        TR_HIP(t, hipMemcpyAsync(d_pre, prefix_occ, n_prefix * 4, hipMemcpyHostToDevice, s));
    }
    if (!d_out) {
        if (pool_malloc(t->ctx, &d_own, t->n * 4 + 4) != hipSuccess) {
            d_own = nullptr;
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "expand: hipMalloc(output) failed");
        }
        d_out = d_own;
    }
    uint64_t tot = 0;
    int rc = t->u16 ? trainer_expand<uint16_t>(t, d_pre ? d_pre : prefix_occ, n_prefix, d_out, &tot)
                    : trainer_expand<uint32_t>(t, d_pre ? d_pre : prefix_occ, n_prefix, d_out, &tot);
    if (rc == GBPE_OK && !out_on_device &&
        (hipMemcpy(out, d_out, t->n * 4, hipMemcpyDeviceToHost) != hipSuccess))
        rc = gbpe_set_error(t->ctx, GBPE_E_DEVICE, "expand: copy to host failed");
    *n_out = tot;
    return rc;
}
