// BPE training merge loop on MI355X (gfx950).
//
// Replaces the reference's 8-dispatch-per-merge WGSL pipeline
// (training-pipeline.js:178-222: clear_table → pair_count_b → find_max_pair4 →
// find_max_pair_final_det → setup_merge → merge_reduce_b → scan_blocks →
// finalize_compact_b, train.wgsl) with an incremental design:
//
//   * the pair-count table PERSISTS across merges; instead of clearing 2^21
//     slots and recounting every pair of the stream each merge
//     (train.wgsl:188-202, 366-431), a merge only emits count deltas at its
//     merge sites, aggregated per workgroup in LDS, then added into the
//     global table — exact counts, no silent drops (train.wgsl:422-429);
//   * argmax is a two-level tournament: per-2048-slot block maxima, only
//     recomputed for blocks a merge touched, then one workgroup reduces them
//     with the reference's tie-break (higher count, then smaller a<<16|b,
//     train.wgsl:83-85);
//   * the stream pass is two streaming kernels over 8192-symbol tiles:
//     k_delta (reads the stream; writes a 1-bit merge-site mask, per-tile
//     survivor counts and count deltas) and k_compact (reads stream + mask,
//     rewrites merged symbols in place, scatters survivors into the
//     ping-pong buffer at a two-level tile prefix).  k_compact never reads a
//     neighbour symbol, so snapshot semantics (train.wgsl:476) hold without
//     the reference's race;
//   * symbols are u16 (bit 15 = word start) whenever every token id fits in
//     15 bits (vocab <= 32768), else u32 with bit 16 (train.wgsl:36-37), so
//     the common 32K-vocab case moves half the bytes.
//
// The reference's compaction quirk (bpe_finalize_compact_b bounded by the
// NEW symbol count, train.wgsl:605-607 + 698/727) is reproduced by default:
// survivors whose old index is >= the new count are not scattered and the
// stale ping-pong contents stay in the stream; k_compact's tail blocks add
// the pairs of that stale window to the count table.
//
// Per merge: k_select (1 WG) → k_delta → k_compact (tiles + tail) → k_refresh.


#include <chrono>
#include "trainer.h"

int trainer_create_impl(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                        int input_on_device, const gbpe_train_opts* opts, uint64_t cap_extra, gbpe_trainer** out,
                        const StateInit* si) {
    if (!ctx || !out || !opts) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *out = nullptr;
    if (n == 0) return gbpe_set_error(ctx, GBPE_E_EMPTY, "No symbols to train on — corpus is empty after pre-processing");
    if (!bytes) return gbpe_set_error(ctx, GBPE_E_INVALID, "bytes is null");
    if (n >= 0xFFFFFFF0ull) return gbpe_set_error(ctx, GBPE_E_INVALID, "corpus too large for one device (%llu symbols)", (unsigned long long)n);
    const auto t_create0 = std::chrono::steady_clock::now();
    auto* t = new (std::nothrow) gbpe_trainer();
    if (!t) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    trainer_config(t, ctx, opts);
    const uint32_t next_id = t->next_id0;
    t->bps = t->u16 ? 2 : 4;
    t->n0 = n;
    t->n = (uint32_t)n;
    hipStream_t s = ctx->stream;
    auto fail = [&](int code) {
        gbpe_trainer_destroy(t);
        return code;
    };
    // buffers padded to whole tiles (+1 tile for the halo / next-word reads); a
    // shard may also grow by appended stale windows (cap_extra symbols)
    if (n + cap_extra >= 0xFFFFFFF0ull - 2 * TILE)
        return fail(gbpe_set_error(ctx, GBPE_E_INVALID, "shard capacity too large for one device"));
    const uint64_t ntiles0 = gbpe_div_up(n + cap_extra, TILE);
    t->cap_syms = (ntiles0 + 1) * TILE;
    for (int k = 0; k < 2; ++k) {
        if (pool_malloc(t->ctx, &t->buf[k], t->cap_syms * t->bps) != hipSuccess)
            return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(symbols) failed"));
        // both ping-pong buffers start zeroed, as WebGPU zero-initialises buffers
        if (hipMemsetAsync(t->buf[k], 0, t->cap_syms * t->bps, s) != hipSuccess)
            return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "memset failed"));
    }
    // pair table
    // distinct pairs start below 65536 (byte pairs) and grow by a few per merge
    // (1 GiB English at 32K: 170K live, 243K slots used): start at 2^20 slots and
    // grow when crowded (trainer_step_once).  An oversized table costs every merge:
    // k_refresh scans one dirty flag per 256-slot block (2^24 slots: 65,536 flags,
    // 1,024 workgroups) and sel_inline reduces one partial maximum per k_refresh
    // workgroup.
    uint32_t lg = opts->table_log2;
    if (lg == 0) lg = 20;
    if (lg < BLK_LOG2 + 1) lg = BLK_LOG2 + 1;
    if (lg > 28) lg = 28;
    t->table_log2 = lg;
    const uint64_t slots = 1ull << lg;
    t->tb.mask = (uint32_t)(slots - 1);
    t->tb.nblk = (uint32_t)(slots >> BLK_LOG2);
    if (pool_malloc(t->ctx, &t->tb.slots, slots * sizeof(uint2)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.bmax, t->tb.nblk * sizeof(uint64_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.bmax2, t->tb.nblk * sizeof(uint64_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.dirty, t->tb.nblk * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.dlist, (t->tb.nblk + 1) * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tb.blive, t->tb.nblk * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->hitmask, (ntiles0 + 1) * TPB * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->tile_cnt, (ntiles0 + 1) * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->grpsum, (ntiles0 / GRP + 2) * GSTR * sizeof(uint32_t)) != hipSuccess ||
        pool_malloc(t->ctx, &t->st, sizeof(DevState)) != hipSuccess ||
        pool_malloc(t->ctx, &t->d_log, (size_t)t->batch * 4 * sizeof(uint32_t)) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(training buffers) failed"));
    if (pool_hmalloc(t->ctx, &t->h_st, sizeof(DevState)) != hipSuccess ||
        pool_hmalloc(t->ctx, &t->h_log, (size_t)t->batch * 4 * sizeof(uint32_t)) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipHostMalloc failed"));
    t->tb.used = &t->st->used;
    t->g_refresh = grid_blocks(ctx, t->tb.nblk, 2);
    if (t->refresh_blocks) t->g_refresh = std::max<uint32_t>(t->refresh_blocks, (uint32_t)gbpe_div_up(t->tb.nblk, 64));
    if (hipMemsetAsync(t->tb.dirty, 0, t->tb.nblk * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(t->hitmask, 0, (ntiles0 + 1) * TPB * sizeof(uint32_t), s) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "memset failed"));
    DevState init{};
    init.n = (uint32_t)n;
    init.next_id = next_id;
    if (si && si->n_prev > n) {   // the last merge's count (the zone rule's mc_prev)
        init.mc = (uint32_t)(si->n_prev - n);
        t->last_mc = init.mc;
        t->n_prev0 = si->n_prev;
    }
    memcpy(t->h_st, &init, sizeof(init));
    if (hipMemcpyAsync(t->st, t->h_st, sizeof(DevState), hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "state upload failed"));
    auto finish = [&]() -> int {
        if (t->flags & GBPE_TRAIN_TIMING) {
            t->evs.resize(5 * t->batch);
            for (auto& e : t->evs)
                if (hipEventCreate(&e) != hipSuccess) return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "hipEventCreate failed"));
        }
        if (hipStreamSynchronize(s) != hipSuccess) return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "trainer init failed"));
        t->ms_create = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_create0).count();
        *out = t;
        return GBPE_OK;
    };
    if (si) {   // both ping-pong buffers from u32 streams (host or device resident)
        const uint32_t* d_cur = (const uint32_t*)bytes;
        const uint32_t* d_prev = si->prev;
        void* tmp = nullptr;
        if (!input_on_device) {
            if (pool_malloc(t->ctx, &tmp, (n + si->n_prev) * 4 + 4) != hipSuccess)
                return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(state) failed"));
            uint32_t* h = (uint32_t*)tmp;
            if (hipMemcpyAsync(h, bytes, n * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
                (si->n_prev && hipMemcpyAsync(h + n, si->prev, si->n_prev * 4, hipMemcpyHostToDevice, s) != hipSuccess)) {
                pool_free(t->ctx, tmp);
                return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "state upload failed"));
            }
            d_cur = h;
            d_prev = h + n;
        }
        auto imp = [&](const uint32_t* src, void* dst, uint64_t cnt) {
            if (!cnt) return;
            const uint32_t g = (uint32_t)gbpe_div_up(cnt, TPB);
            if (t->u16)
                hipLaunchKernelGGL(k_import_symbols<uint16_t>, dim3(g), dim3(TPB), 0, s, src, (uint16_t*)dst, cnt);
            else
                hipLaunchKernelGGL(k_import_symbols<uint32_t>, dim3(g), dim3(TPB), 0, s, src, (uint32_t*)dst, cnt);
        };
        imp(d_cur, t->buf[0], n);
        if (d_prev) imp(d_prev, t->buf[1], si->n_prev);
        const bool launched = hipGetLastError() == hipSuccess;
        int rc = launched ? table_rebuild(t) : gbpe_set_error(ctx, GBPE_E_DEVICE, "symbol import launch failed");
        hipStreamSynchronize(s);
        pool_free(t->ctx, tmp);
        if (rc != GBPE_OK) return fail(rc);
        return finish();
    }
    // symbols: bytes (+ mask) → S with word-start bit; input may be host or device resident
    const uint8_t* d_bytes = bytes;
    const uint8_t* d_ws = word_starts;
    void* tmp = nullptr;
    if (!input_on_device) {
        const uint64_t need = n * (word_starts ? 2 : 1);
        if (pool_malloc(t->ctx, &tmp, need) != hipSuccess) return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(input) failed"));
        if (hipMemcpyAsync(tmp, bytes, n, hipMemcpyHostToDevice, s) != hipSuccess ||
            (word_starts && hipMemcpyAsync((uint8_t*)tmp + n, word_starts, n, hipMemcpyHostToDevice, s) != hipSuccess)) {
            pool_free(t->ctx, tmp);
            return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "input upload failed"));
        }
        d_bytes = (const uint8_t*)tmp;
        d_ws = word_starts ? (const uint8_t*)tmp + n : nullptr;
    }
    uint8_t* d_gpt4 = nullptr;   // GPT-4 rule word starts computed on the device (pre_tokenizer.mjs:226-292)
    if (!d_ws && (opts->flags & GBPE_TRAIN_GPT4_BOUNDARIES)) {
        int rc2 = pool_malloc(t->ctx, &d_gpt4, n) == hipSuccess ? gbpe_pretok_gpt4_launch(ctx, d_bytes, n, d_gpt4) : GBPE_E_OOM;
        if (rc2 != GBPE_OK) {
            if (tmp) pool_free(t->ctx, tmp);
            pool_free(t->ctx, d_gpt4);
            return fail(rc2 == GBPE_E_OOM ? gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(word starts) failed") : rc2);
        }
        d_ws = d_gpt4;
    }
    const uint32_t gb = (uint32_t)gbpe_div_up(n, TPB);
    const bool vec = ((uintptr_t)d_bytes & 15u) == 0 && ((uintptr_t)d_ws & 15u) == 0;   // (null is aligned)
    const uint32_t gv = (uint32_t)gbpe_div_up(gbpe_div_up(n, 16), TPB);
    if (t->u16 && vec)
        hipLaunchKernelGGL(k_symbols_v<uint16_t>, dim3(gv), dim3(TPB), 0, s, d_bytes, d_ws, (uint16_t*)t->buf[0], n);
    else if (vec)
        hipLaunchKernelGGL(k_symbols_v<uint32_t>, dim3(gv), dim3(TPB), 0, s, d_bytes, d_ws, (uint32_t*)t->buf[0], n);
    else if (t->u16)
        hipLaunchKernelGGL(k_symbols<uint16_t>, dim3(gb), dim3(TPB), 0, s, d_bytes, d_ws, (uint16_t*)t->buf[0], n,
                           (uint8_t*)nullptr);
    else
        hipLaunchKernelGGL(k_symbols<uint32_t>, dim3(gb), dim3(TPB), 0, s, d_bytes, d_ws, (uint32_t*)t->buf[0], n,
                           (uint8_t*)nullptr);
    if (hipGetLastError() != hipSuccess) {
        if (tmp) pool_free(t->ctx, tmp);
        return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "symbol kernel launch failed"));
    }
    int rc = table_rebuild(t, true);
    if (tmp || d_gpt4) {
        hipStreamSynchronize(s);
        pool_free(t->ctx, tmp);
        pool_free(t->ctx, d_gpt4);
    }
    if (rc != GBPE_OK) return fail(rc);
    return finish();
}

extern "C" int gbpe_trainer_create(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                                   int input_on_device, const gbpe_train_opts* opts, gbpe_trainer** out) {
    return trainer_create_impl(ctx, bytes, n, word_starts, input_on_device, opts, 0, out);
}

extern "C" int gbpe_trainer_create_from_state(gbpe_ctx* ctx, const uint32_t* cur, uint64_t n, const uint32_t* prev,
                                              uint64_t n_prev, int input_on_device, const gbpe_train_opts* opts,
                                              gbpe_trainer** out) {
    if (n_prev < n) return gbpe_set_error(ctx, GBPE_E_INVALID, "create_from_state: n_prev (%llu) < n (%llu)",
                                          (unsigned long long)n_prev, (unsigned long long)n);
    if (n_prev > n && !prev) return gbpe_set_error(ctx, GBPE_E_INVALID, "create_from_state: prev is null");
    const StateInit si{prev, n_prev};
    return trainer_create_impl(ctx, (const uint8_t*)cur, n, nullptr, input_on_device, opts, n_prev - n, out, &si);
}

namespace {
int trainer_step_once(gbpe_trainer* t, uint32_t max_merges, uint32_t* merges_out, uint32_t* n_done, uint32_t* early_stop) {
    const auto hs0 = std::chrono::steady_clock::now();
    if (t->htime && t->ht_steps) t->ht_out += std::chrono::duration<double, std::micro>(hs0 - t->ht_last).count();
    if (n_done) *n_done = 0;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    uint32_t k = max_merges ? max_merges : t->batch;
    if (k > t->batch) k = t->batch;
    if (t->done + k > t->needed) k = t->needed - t->done;
    if (t->stop || k == 0) return GBPE_OK;
    hipStream_t s = t->ctx->stream;
    // rebuild the pair table when it gets crowded (dead pairs accumulate), twice as
    // large (or more) while the live pairs would fill over a quarter of it
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    if ((uint64_t)t->h_st->used * 100 > slots * t->grow_used_pct) {
        const uint64_t live = std::max<uint64_t>(t->h_st->live, t->h_st->used / 2);
        uint32_t lg = t->table_log2;
        while (lg < 28 && live * 100 > (1ull << lg) * t->grow_live_pct) ++lg;
        int rc;
        if (t->sp && t->rehash_on) {   // the sparse loop goes on over the moved entries
            rc = table_rehash(t, lg);
        } else {
            rc = sp_exit_any(t);   // the full recount runs on the dense stream
            if (rc == GBPE_OK && lg != t->table_log2) rc = table_resize(t, lg);
            if (rc == GBPE_OK) rc = table_rebuild(t);
        }
        if (rc != GBPE_OK) return rc;
        ++t->table_grows;
    }
    // sector-sparse loop once merges touch a small fraction of the stream
    if (t->sp_cooldown) {
        --t->sp_cooldown;
    } else if (!t->sp && !(t->flags & GBPE_TRAIN_DENSE_ONLY)) {
        // with the word lexicon the body costs what its distinct words cost, so the
        // loop can enter as soon as the zone (~7 x the next count) is a small part of
        // the stream — before the first merge; without it, once counts
        // are a 1/sp_div fraction
        // with the lexicon the decision (and the zone) follow the NEXT merge's count,
        // the table maximum: one huge first merge (C5's (32,32), 17 % of the stream)
        // then ends only a one-merge dense step (enter_lim below)
        uint32_t mc = t->last_mc, next = 0;
        if (t->lex_on) {
            if (!t->d_u32) TR_HIP(t, pool_malloc(t->ctx, &t->d_u32, 64));
            hipLaunchKernelGGL(k_topcount, dim3(1), dim3(1024), 0, s, t->tb, t->d_u32);
            GBPE_LAUNCH_CHECK(t->ctx);
            TR_HIP(t, hipMemcpyAsync(&next, t->d_u32, 4, hipMemcpyDeviceToHost, s));
            TR_HIP(t, hipStreamSynchronize(s));
            mc = next;
        }
        const uint64_t div = t->lex_on ? t->lx_div : t->sp_div;
        const bool count_ok = mc && ((t->flags & GBPE_TRAIN_SPARSE_EARLY) || (uint64_t)mc * div <= t->n);
        if (count_ok) {
            int rc = t->u16 ? sp_enter<uint16_t>(t, true, next) : sp_enter<uint32_t>(t, true, next);
            if (rc != GBPE_OK) return rc;
        }
        // still dense with the lexicon on: the device ends the step once a merge's count
        // would pass the entry test, so the loop enters at the next step boundary
        const uint32_t lim = (!t->sp && t->lex_on && mc && !count_ok) ? (uint32_t)(t->n / div) : 0u;
        if (lim != t->h_st->enter_lim) {
            t->h_st->enter_lim = lim;
            TR_HIP(t, hipMemcpyAsync(&t->st->enter_lim, &t->h_st->enter_lim, sizeof(uint32_t), hipMemcpyHostToDevice, s));
        }
    }
    // keep the zone near its minimum, then rebuild stale filters now and then
    if (t->sp) {
        const auto a0 = std::chrono::steady_clock::now();
        const uint32_t ns0 = t->sp_shrinks;
        int rc = t->u16 ? sp_shrink<uint16_t>(t) : sp_shrink<uint32_t>(t);
        if (rc != GBPE_OK) return rc;
        if (t->htime && t->sp_shrinks != ns0) {
            t->ht_shrink += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a0).count();
            ++t->ht_nshrink;
        }
    }
    if (t->sp && t->sp_age >= 4096) {   // signatures saturate faster than the token bitmap goes stale
        const auto a0 = std::chrono::steady_clock::now();
        const bool wb = t->sp_bits_age >= 16384;
        int rc = t->u16 ? sp_filters<uint16_t>(t, wb) : sp_filters<uint32_t>(t, wb);
        if (rc != GBPE_OK) return rc;
        if (t->htime) {
            t->ht_filters += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a0).count();
            ++t->ht_nfilters;
        }
    }
    // waiting for the lexicon entry on a long stream: one merge per step (a dense merge
    // costs milliseconds there; every round the step enqueues after the entry point
    // would still launch its full-grid kernels as no-ops)
    if (!t->sp && t->h_st->enter_lim && t->n >= (1u << 24)) k = 1;
    // a large zone shrinks every sub_k merges instead of every step (early counts fall fast)
    if (t->sp && (uint32_t)t->n - t->h_st->B > t->sub_zone && k > t->sub_k) k = t->sub_k;
    // reset the per-step counter + budget (trainer.js:239)
    DevState* hs = t->h_st;
    hs->merges_done = 0;
    hs->budget = k;
    if (t->sp) hs->sel_round = 0;
    hipLaunchKernelGGL(k_step_in, dim3(1), dim3(1), 0, s, t->st, t->sp ? t->zst : (DevState*)nullptr, k);
#ifdef GBPE_KTRACE
    if (getenv("GBPE_KTRACE_OUT")) {
        static unsigned long long* kbuf = nullptr;
        if (!kbuf) {
            const size_t nb = (size_t)(KT_MERGES / KT_EVERY) * 2 * KT_WG * KT_SLOTS * 8;
            TR_HIP(t, pool_malloc(t->ctx, &kbuf, nb));
            TR_HIP(t, hipMemsetAsync(kbuf, 0, nb, s));
            TR_HIP(t, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ktr), &kbuf, sizeof(kbuf), 0, hipMemcpyHostToDevice, s));
        }
        const uint32_t kb = (uint32_t)t->done;
        TR_HIP(t, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_kt_base), &kb, 4, 0, hipMemcpyHostToDevice, s));
    }
#endif
    const uint64_t ntiles = gbpe_div_up(t->n, TILE);
    // tile blocks + stale-tail blocks (the window is at most mc <= n/2 symbols)
    const uint32_t g_tail = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u
                            : grid_persistent(t->ctx, gbpe_div_up(t->n / 2 + 1, TPB * 16), 1);
    const uint32_t g_delta = (uint32_t)(ntiles ? ntiles : 1);
    const uint32_t g_compact = (uint32_t)ntiles + g_tail;
    uint32_t g_refresh = t->g_refresh;
    const bool timing = (t->flags & GBPE_TRAIN_TIMING) != 0;
    const bool sparse = t->sp;
    SpGrid sg{};
    if (sparse) {
        const uint32_t zn = (uint32_t)t->n - hs->B;   // zone length (it only shrinks within a step)
        const uint64_t zt = gbpe_div_up(zn, TILE);
        const uint32_t z256 = t->u16 ? zone_max<uint16_t>(256) : zone_max<uint32_t>(256);
        sg.bt = zn <= std::min<uint32_t>(z256, t->z256) ? 256 : 1024;   // small zone: the low-latency 256-thread workgroups
        body_grid(t, sg.bt, &sg.body, &sg.wpg, 0, &sg.sub);
        if (sg.bt == 1024 && t->u16 && zn <= 16384u && t->zone16) sg.bt = 1023;
        sg.zone1 = zn <= (t->u16 ? zone_max<uint16_t>(sg.bt) : zone_max<uint32_t>(sg.bt)) ? 1u : 0u;
        // a zone of 16K-1M symbols: 16K-symbol segments inside k_body (its ZSEG form)
        const uint32_t zs_lo = t->zseg_mode == 2 ? (t->u16 ? zone_max<uint16_t>(1024) : zone_max<uint32_t>(1024)) : t->zseg_lo;
        if (t->zseg_mode && t->zseg && zn > zs_lo && zn <= NSEG_MAX * 16384u) {
            sg.seg8 = t->seg8 && zn <= NSEG_MAX * 8192u;
            sg.zone1 = (uint32_t)gbpe_div_up(zn, sg.seg8 ? 8192u : 16384u);
        }
        sg.copy = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u : grid_persistent(t->ctx, gbpe_div_up(zn / 5 + 1, TPB * 8), 1);
        sg.zdelta = (uint32_t)(zt ? zt : 1);
        sg.ztail = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u
                                                           : (uint32_t)std::min<uint64_t>(1024, gbpe_div_up(zn / 5 + 1, 2048));
        sg.zcompact = (uint32_t)zt + ((t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u
                                      : grid_persistent(t->ctx, gbpe_div_up(zn / 2 + 1, TPB * 16), 1));
        // the 1024-thread forms hold one workgroup per CU (their LDS): the zone's (or
        // the window copy's) workgroups beside the body's, past the CU count, wait for
        // a CU to drain (C5 merges 512-8K: the last one started 14-19 us late) — so
        // the body takes the CUs the others leave
        const uint32_t extra = sg.zone1 ? sg.zone1 : sg.copy;
        if (sg.bt >= 1023 && t->body_fit && extra && sg.body + extra > t->body_cap && 2 * extra <= t->body_cap)
            body_grid(t, sg.bt, &sg.body, &sg.wpg, t->body_cap - extra, &sg.sub);
        // late steps (a zone of <= 16K symbols): a smaller k_refresh grid —
        // a late merge dirties a few blocks, and fewer workgroups dispatch and drain
        // sooner.  The partial maxima the next k_body reads are laid out per k_refresh
        // workgroup, so a grid change re-lays them out once (finish 0: no merge closed)
        if (t->refresh_late && zn <= t->refresh_late_z) {
            // (at most one workgroup per block: the partial maxima hold nblk + 1 per half;
            // at most TPB blocks per workgroup)
            const uint32_t want = std::min<uint32_t>(t->tb.nblk,
                                                     std::max<uint32_t>(t->refresh_late, (uint32_t)gbpe_div_up(t->tb.nblk, TPB)));
            if (want != t->g_refresh) {
                t->g_refresh = g_refresh = want;
                if (t->u16)
                    GBPE_LAUNCH_REFRESH(uint16_t, want, t->tb.nblk, s, t->st, 0u, 0, t->tb, (uint16_t*)nullptr,
                                        (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(),
                                        t->part, (uint32_t*)nullptr);
                else
                    GBPE_LAUNCH_REFRESH(uint32_t, want, t->tb.nblk, s, t->st, 0u, 0, t->tb, (uint32_t*)nullptr,
                                        (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(),
                                        t->part, (uint32_t*)nullptr);
                GBPE_LAUNCH_CHECK(t->ctx);
            }
        }
        sg.refresh = g_refresh;
        // paired launches: the late zone_one form, two merges per launch
        // when the table's top two allow it
        sg.pair = t->pair_on && sg.zone1 == 1 && sg.bt == 256 && t->zseg && k >= 2;
    }
    // a paired step needs fewer launches than merges: sized by the last paired step's
    // rate (+2); launches past the step's budget are no-ops, and a step whose launches
    // ran out first is continued by gbpe_trainer_step
    uint32_t nl = k;
    if (sg.pair) nl = std::min<uint32_t>(k, (uint32_t)std::ceil((double)k / (1.0 + t->pair_rate)) + 2u);
    const uint32_t paired0 = hs->paired;
    auto launch_all = [&]() -> int {
        for (uint32_t r = 0; r < nl; ++r) {
            hipEvent_t* ev = timing ? &t->evs[5 * r] : nullptr;
            int rc;
            if (sparse)
                rc = t->u16 ? launch_merge_sparse<uint16_t>(t, r, s, sg, timing, ev)
                            : launch_merge_sparse<uint32_t>(t, r, s, sg, timing, ev);
            else
                rc = t->u16 ? launch_merge<uint16_t>(t, r, s, g_delta, g_compact, g_refresh, timing, ev)
                            : launch_merge<uint32_t>(t, r, s, g_delta, g_compact, g_refresh, timing, ev);
            if (rc != GBPE_OK) return rc;
        }
        return GBPE_OK;
    };
    const auto h0 = std::chrono::steady_clock::now();
    auto h1 = h0;
    {
        int rc = launch_all();
        if (rc != GBPE_OK) return rc;
        h1 = std::chrono::steady_clock::now();
        // the read-backs (and, sparse, k_live's count) in one launch: no copy blits
        const bool cl = sparse && t->d_clog;
        hipLaunchKernelGGL(k_step_out, dim3(1), dim3(1024), 0, s, t->st, sparse ? t->zst : (DevState*)nullptr, t->tb,
                           sparse ? 1 : 0, (const uint32_t*)t->d_log, k * 4u, (const uint32_t*)(cl ? t->d_clog : nullptr),
                           cl ? k * 2u : 0u, t->h_st, t->h_zst, t->h_log, cl ? t->h_clog : (uint32_t*)nullptr);
        GBPE_LAUNCH_CHECK(t->ctx);
    }
    TR_HIP(t, hipStreamSynchronize(s));
    const uint32_t done = hs->merges_done;
    {
        const uint32_t dbl = hs->paired - paired0;   // launches that ran two merges
        t->pair_done += dbl;
        if (sg.pair && done > dbl) t->pair_rate = (double)dbl / (double)(done - dbl);
        if (t->ptrace)   // (diagnostic, GBPE_DEBUG ptrace=1) the step's form and pairing
            fprintf(stderr, "[ptrace] merge %u zone %u zone1 %u bt %d pair %d launches %u done %u paired %u cand %u mc %u us %.1f\n",
                    t->done, hs->n - hs->B, sg.zone1, sg.bt, sg.pair ? 1 : 0, nl, done, dbl,
                    hs->pair_cand, done ? t->h_log[(done - 1) * 4 + 3] : 0u,
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - hs0).count());
    }
    if (t->htime) {   // (diagnostic) host enqueue vs wait; "late": a zone of <= 16K symbols
        t->ht_pre += std::chrono::duration<double, std::micro>(h0 - hs0).count();
        const double enq = std::chrono::duration<double, std::micro>(h1 - h0).count();
        const double wait = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h1).count();
        t->ht_enq += enq;
        t->ht_wait += wait;
        ++t->ht_steps;
        if (sparse && (uint32_t)t->n - hs->B <= 16384u) {
            t->ht_enq_late += enq;
            t->ht_wait_late += wait;
            ++t->ht_steps_late;
            t->ht_merges_late += done;
        }
    }
#ifdef GBPE_BSPROF
    if (sparse && getenv("GBPE_BSPROF")) {   // body_sector's cycle split of this step (train_dev.h)
        unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        TR_HIP(t, hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bsprof), sizeof(h), 0, hipMemcpyDeviceToHost));
        fprintf(stderr, "[bsprof] merges %u-%u waves %llu sectors %llu passes %llu | cyc/sector loads+hits %.0f deltas %.0f "
                        "writes %.0f flush %.0f | sector-phase cyc/wave %.0f\n",
                (unsigned)t->done, (unsigned)(t->done + done), h[7], h[5], h[4], h[5] ? (double)h[0] / h[5] : 0.0,
                h[5] ? (double)h[1] / h[5] : 0.0, h[5] ? (double)h[2] / h[5] : 0.0, h[5] ? (double)h[3] / h[5] : 0.0,
                h[7] ? (double)h[6] / h[7] : 0.0);
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        TR_HIP(t, hipMemcpyToSymbol(HIP_SYMBOL(g_bsprof), z, sizeof(z), 0, hipMemcpyHostToDevice));
    }
#endif
    const uint32_t err = hs->err | (sparse ? t->h_zst->err : 0u);
    if (err) {
        return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "training invariant violated (err=0x%x: %s%s%s%s%s)", err,
                              (err & ERR_TABLE_FULL) ? "pair table full " : "",
                              (err & ERR_COUNT_MISMATCH) ? "survivor count mismatch " : "",
                              (err & ERR_PAIR_MISSING) ? "selected pair missing " : "",
                              (err & ERR_SPARSE_WINDOW) ? "sparse stale window outside the zone " : "",
                              (err & ERR_SPIN) ? "zone segment hand-off timed out" : "");
    }
    if (timing) {
        for (uint32_t r = 0; r < std::min(done, nl); ++r) {   // (per launch)
            float a = 0, b = 0, c = 0, d1 = 0, d2 = 0;
            hipEvent_t* ev = &t->evs[5 * r];
            hipEventElapsedTime(&a, ev[0], ev[1]);
            hipEventElapsedTime(&b, ev[1], ev[2]);
            hipEventElapsedTime(&c, ev[2], ev[4]);
            hipEventElapsedTime(&d1, ev[1], ev[3]);
            hipEventElapsedTime(&d2, ev[3], ev[2]);
            t->ms_select += a;
            t->ms_merge += b;
            t->ms_other += c;
            t->ms_delta += d1;
            t->ms_compact += d2;
            (sparse ? t->ms_sparse : t->ms_dense) += b;
            if (sparse) t->ms_body += d1;
        }
        t->timed_merges += done;
    }
    // algorithmic stream bytes: s * (2 N_i + N_{i+1})
    uint64_t N = t->n;
    for (uint32_t r = 0; r < done; ++r) {
        const uint64_t mc = t->h_log[r * 4 + 3];
        t->bytes_moved += (uint64_t)t->bps * (2 * N + (N - mc));
        if (!sparse) t->dense_bytes += (uint64_t)t->bps * (2 * N + (N - mc));
        N -= mc;
        if (merges_out) memcpy(merges_out + 4 * r, t->h_log + 4 * r, 4 * sizeof(uint32_t));
    }
    if ((uint32_t)N != hs->n) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "host/device symbol count disagree");
    t->n = N;
    if (done) t->last_mc = t->h_log[(done - 1) * 4 + 3];
    if (t->trace) {   // merge index, count, stream length before, sparse, candidate sectors, sectors with sites
        uint64_t nn = N;
        for (uint32_t r = done; r-- > 0;) nn += t->h_log[r * 4 + 3];
        for (uint32_t r = 0; r < done; ++r) {
            fprintf(t->trace, "%u %u %llu %d %u %u\n", t->done + r, t->h_log[r * 4 + 3], (unsigned long long)nn,
                    sparse ? 1 : 0, sparse && t->h_clog ? t->h_clog[2 * r] : 0u, sparse && t->h_clog ? t->h_clog[2 * r + 1] : 0u);
            nn -= t->h_log[r * 4 + 3];
        }
    }
    if (sparse) {
        t->zcur ^= (int)(done & 1u);
        t->sp_merges += done;
        t->sp_age += done;
        t->sp_bits_age += done;
        if (hs->sp_abort) {   // a merge outgrew the zone: it was not run; continue dense
            int rc = sp_exit_any(t);
            if (rc != GBPE_OK) return rc;
            t->sp_cooldown = 1;
            if (done == 0 && !hs->stop) return trainer_step_once(t, max_merges, merges_out, n_done, early_stop);
        }
    } else {
        t->cur ^= (done & 1u);
    }
    t->done += done;
    t->stop = hs->stop != 0;
    if (n_done) *n_done = done;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    if (t->htime) {
        t->ht_last = std::chrono::steady_clock::now();
        t->ht_post += std::chrono::duration<double, std::micro>(t->ht_last - h1).count();
    }
    return GBPE_OK;
}
}  // namespace

// One host step of up to max_merges merges (trainer.js:225-335's 128-merge batch).
// Internally a sparse step whose zone is still large runs as several sub-steps
// (trainer_step_once), so the zone can shrink between them.
extern "C" int gbpe_trainer_step(gbpe_trainer* t, uint32_t max_merges, uint32_t* merges_out, uint32_t* n_done,
                                 uint32_t* early_stop) {
    if (!t) return GBPE_E_INVALID;
    uint32_t want = max_merges ? max_merges : t->batch;
    if (want > t->batch) want = t->batch;
    uint32_t got = 0, es = 0;
    int rc = GBPE_OK;
    while (got < want) {
        uint32_t nd = 0;
        rc = trainer_step_once(t, want - got, merges_out ? merges_out + 4 * got : nullptr, &nd, &es);
        if (rc != GBPE_OK) break;
        got += nd;
        if (nd == 0 || es) break;
    }
    if (n_done) *n_done = got;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    return rc;
}

extern "C" int gbpe_trainer_stats_get(gbpe_trainer* t, gbpe_trainer_stats* o) {
    if (!t || !o) return GBPE_E_INVALID;
    memset(o, 0, sizeof(*o));
    o->symbol_count = t->n;
    o->merges_done = t->done;
    o->stream_bytes_moved = t->bytes_moved;
    o->tail_dropped = t->h_st->tail_total;
    o->table_slots = (uint64_t)t->tb.mask + 1;
    o->table_used = t->h_st->used;
    o->bytes_per_symbol = t->bps;
    o->early_stop = t->stop;
    o->ms_merge = t->ms_merge;
    o->ms_delta = t->ms_delta;
    o->ms_compact = t->ms_compact;
    o->ms_select = t->ms_select;
    o->ms_other = t->ms_other;
    o->timed_merges = t->timed_merges;
    o->live_pairs = t->h_st->live;
    o->max_live_pairs = t->h_st->max_live;
    o->sparse_merges = t->sp_merges;
    o->sparse_enters = t->sp_enters;
    o->sparse_exits = t->sp_exits;
    o->sparse_sectors = t->sp_sectors;
    o->sparse_zone = t->sp_zone;
    o->dense_bytes = t->dense_bytes;
    o->ms_dense = t->ms_dense;
    o->ms_sparse = t->ms_sparse;
    o->ms_body = t->ms_body;
    o->ms_create = t->ms_create;
    o->paired_merges = t->pair_done;
    o->zone_bytes = t->h_st->sp_bytes;
    o->lexicon_builds = (uint32_t)t->lx_builds;
    o->lexicon_fallbacks = (uint32_t)t->lx_fallbacks;
    o->lexicon_words = t->lx_words;
    o->lexicon_entries = t->lx_nuid;
    o->lexicon_symbols = t->lx_len;
    if (t->wg_bytes && t->wg_cap) {   // the per-workgroup counters of k_body (and its zone workgroup)
        std::vector<uint64_t> h(t->wg_cap);
        if (hipMemcpy(h.data(), t->wg_bytes, t->wg_cap * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess)
            for (uint64_t v : h) o->body_bytes += v;
    }
    return GBPE_OK;
}

extern "C" int gbpe_trainer_symbols(gbpe_trainer* t, uint32_t* out, uint64_t cap, uint64_t* n) {
    if (!t || !n) return GBPE_E_INVALID;
    *n = t->n;
    if (!out) return GBPE_OK;
    if (cap < t->n) return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "symbols: need %llu", (unsigned long long)t->n);
    {
        int rc = sp_exit_any(t);   // back to one dense stream (training may go on; it re-enters later)
        if (rc != GBPE_OK) return rc;
    }
    hipStream_t s = t->ctx->stream;
    uint32_t* d = nullptr;
    TR_HIP(t, pool_malloc(t->ctx, &d, (uint64_t)t->n * 4 + 4));
    const uint32_t g = (uint32_t)gbpe_div_up(t->n, 256);
    if (t->n) {
        if (t->u16)
            hipLaunchKernelGGL(k_export_symbols<uint16_t>, dim3(g), dim3(256), 0, s, (const uint16_t*)t->buf[t->cur], d,
                               (uint64_t)t->n);
        else
            hipLaunchKernelGGL(k_export_symbols<uint32_t>, dim3(g), dim3(256), 0, s, (const uint32_t*)t->buf[t->cur], d,
                               (uint64_t)t->n);
    }
    hipError_t e = hipMemcpyAsync(out, d, (uint64_t)t->n * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    pool_free(t->ctx, d);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "symbol export failed: %s", hipGetErrorString(e));
    return GBPE_OK;
}

// current + previous stream (consolidation).  The previous stream
// is the other ping-pong buffer over the previous length:
// n + last count on one device (zeros before the first merge).
extern "C" int gbpe_trainer_export_state(gbpe_trainer* t, uint32_t* cur, uint64_t cap_cur, uint64_t* n_cur,
                                         uint32_t* prev, uint64_t cap_prev, uint64_t* n_prev, int on_device) {
    if (!t || !n_cur || !n_prev) return GBPE_E_INVALID;
    {
        int rc = sp_exit_any(t);   // one dense stream (+ its stale buffer where the next window can read)
        if (rc != GBPE_OK) return rc;
    }
    hipStream_t s = t->ctx->stream;
    TR_HIP(t, hipMemcpyAsync(t->h_st, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    const uint64_t n = t->n;
    // (a trainer created from a state and not stepped since re-exports the imported length)
    uint64_t np = t->done ? n + t->last_mc : (t->n_prev0 ? t->n_prev0 : n);
    if (np > t->cap_syms) np = t->cap_syms;
    *n_cur = n;
    *n_prev = np;
    if (!cur && !prev) return GBPE_OK;
    if ((cur && cap_cur < n) || (prev && cap_prev < np))
        return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "export_state: need %llu + %llu", (unsigned long long)n,
                              (unsigned long long)np);
    uint32_t* d = nullptr;
    if (!on_device) TR_HIP(t, pool_malloc(t->ctx, &d, (n + np) * 4 + 4));
    auto exp = [&](const void* src, uint32_t* dst, uint64_t cnt) {
        if (!cnt || !dst) return;
        const uint32_t g = (uint32_t)gbpe_div_up(cnt, 256);
        if (t->u16)
            hipLaunchKernelGGL(k_export_symbols<uint16_t>, dim3(g), dim3(256), 0, s, (const uint16_t*)src, dst, cnt);
        else
            hipLaunchKernelGGL(k_export_symbols<uint32_t>, dim3(g), dim3(256), 0, s, (const uint32_t*)src, dst, cnt);
    };
    exp(t->buf[t->cur], on_device ? cur : d, n);
    exp(t->buf[t->cur ^ 1], on_device ? prev : d + n, np);
    hipError_t e = hipGetLastError();
    if (!on_device) {
        if (e == hipSuccess && cur && n) e = hipMemcpyAsync(cur, d, n * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && prev && np) e = hipMemcpyAsync(prev, d + n, np * 4, hipMemcpyDeviceToHost, s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    pool_free(t->ctx, d);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "state export failed: %s", hipGetErrorString(e));
    return GBPE_OK;
}

extern "C" int gbpe_trainer_pair_counts(gbpe_trainer* t, uint32_t* pids, uint32_t* counts, uint64_t cap, uint64_t* n) {
    if (!t || !n) return GBPE_E_INVALID;
    hipStream_t s = t->ctx->stream;
    uint32_t* d = nullptr;
    const uint64_t c = cap ? cap : 1;
    TR_HIP(t, pool_malloc(t->ctx, &d, (2 * c + 1) * sizeof(uint32_t)));
    hipError_t e = hipMemsetAsync(d, 0, sizeof(uint32_t), s);
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    hipLaunchKernelGGL(k_dump_pairs, dim3((uint32_t)gbpe_div_up(slots, 256)), dim3(256), 0, s, t->tb, d + 1, d + 1 + c,
                       d, (uint32_t)cap);
    uint32_t cnt = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&cnt, d, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess && cnt <= cap && cap) {
        e = hipMemcpy(pids, d + 1, (uint64_t)cnt * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(counts, d + 1 + c, (uint64_t)cnt * 4, hipMemcpyDeviceToHost);
    }
    pool_free(t->ctx, d);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "pair dump failed: %s", hipGetErrorString(e));
    *n = cnt;
    if (cnt > cap) return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "pair dump: need %u", cnt);
    return GBPE_OK;
}

extern "C" void gbpe_trainer_destroy(gbpe_trainer* t) {
    if (!t) return;
    if (t->ctx && t->ctx->stream) hipStreamSynchronize(t->ctx->stream);
    if (t->htime && t->h_st)   // paired launches: candidates, window-check rejections, run
        fprintf(stderr, "[pair] candidates %u rejected %u paired %u\n", t->h_st->pair_cand, t->h_st->pair_rej,
                t->h_st->paired);
    if (t->htime && t->ht_steps)
        fprintf(stderr, "[htime] steps %llu: before launch %.2f ms, enqueue %.2f ms, wait %.2f ms, after sync %.2f ms, "
                        "caller between steps %.2f ms, shrinks %llu in %.2f ms, filter rebuilds %llu in %.2f ms | late steps %llu (%llu merges): enqueue %.2f ms "
                        "(%.2f us/merge), wait %.2f ms (%.2f us/merge)\n",
                (unsigned long long)t->ht_steps, t->ht_pre / 1e3, t->ht_enq / 1e3, t->ht_wait / 1e3,
                (t->ht_post - t->ht_wait) / 1e3, t->ht_out / 1e3, (unsigned long long)t->ht_nshrink, t->ht_shrink / 1e3,
                (unsigned long long)t->ht_nfilters, t->ht_filters / 1e3, (unsigned long long)t->ht_steps_late,
                (unsigned long long)t->ht_merges_late, t->ht_enq_late / 1e3,
                t->ht_merges_late ? t->ht_enq_late / t->ht_merges_late : 0.0, t->ht_wait_late / 1e3,
                t->ht_merges_late ? t->ht_wait_late / t->ht_merges_late : 0.0);
#ifdef GBPE_KTRACE
    if (const char* path = getenv("GBPE_KTRACE_OUT")) {   // one file per trainer: path.<done merges>
        std::vector<unsigned long long> h((size_t)(KT_MERGES / KT_EVERY) * 2 * KT_WG * KT_SLOTS);
        unsigned long long* kbuf = nullptr;
        if (hipMemcpyFromSymbol(&kbuf, HIP_SYMBOL(g_ktr), sizeof(kbuf), 0, hipMemcpyDeviceToHost) == hipSuccess && kbuf &&
            hipMemcpy(h.data(), kbuf, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            char fn[512];
            snprintf(fn, sizeof(fn), "%s.%llu", path, (unsigned long long)t->done);
            if (FILE* f = fopen(fn, "wb")) {
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
        if (kbuf) hipMemset(kbuf, 0, h.size() * 8);
    }
#endif
    for (auto& e : t->evs)
        if (e) hipEventDestroy(e);
    pool_free(t->ctx, t->buf[0]);
    pool_free(t->ctx, t->buf[1]);
    pool_free(t->ctx, t->tb.slots);
    pool_free(t->ctx, t->tb.bmax);
    pool_free(t->ctx, t->tb.bmax2);
    pool_free(t->ctx, t->tb.dirty);
    pool_free(t->ctx, t->tb.dlist);
    pool_free(t->ctx, t->tb.blive);
    pool_free(t->ctx, t->hitmask);
    pool_free(t->ctx, t->tile_cnt);
    pool_free(t->ctx, t->grpsum);
    pool_free(t->ctx, t->sec);
    pool_free(t->ctx, t->sp_loc);
    pool_free(t->ctx, t->sp_blk);
    pool_free(t->ctx, t->bits);
    pool_free(t->ctx, t->sig);
    pool_free(t->ctx, t->zbuf[0]);
    pool_free(t->ctx, t->zbuf[1]);
    pool_free(t->ctx, t->wtmp);
    pool_free(t->ctx, t->zst);
    pool_free(t->ctx, t->d_u32);
    pool_free(t->ctx, t->part);
    pool_free(t->ctx, t->d_bhist);
    pool_free(t->ctx, t->zseg);
    pool_free(t->ctx, t->zdr_out);
    pool_free(t->ctx, t->zdr_offs);
    pool_free(t->ctx, t->zdr_flag);
    pool_free(t->ctx, t->wg_bytes);
    pool_free(t->ctx, t->lx_store);
    pool_free(t->ctx, t->lx_mul);
    pool_free(t->ctx, t->lx_occ);
    pool_free(t->ctx, t->lx_w0);
    pool_free(t->ctx, t->lx_tmp);
    if (t->h_zst) pool_hfree(t->ctx, t->h_zst);
    pool_free(t->ctx, t->d_clog);
    if (t->h_clog) pool_hfree(t->ctx, t->h_clog);
    if (t->trace) fclose(t->trace);
    pool_free(t->ctx, t->st);
    pool_free(t->ctx, t->d_log);
    if (t->h_st) pool_hfree(t->ctx, t->h_st);
    if (t->h_log) pool_hfree(t->ctx, t->h_log);
    delete t;
}

extern "C" int gbpe_train(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                          const gbpe_train_opts* opts, gbpe_progress_cb cb, void* user, uint32_t* merges_out,
                          uint32_t merges_cap, uint32_t* n_merges, uint32_t* early_stop) {
    if (n_merges) *n_merges = 0;
    if (early_stop) *early_stop = 0;
    gbpe_trainer* t = nullptr;
    int rc = gbpe_trainer_create(ctx, bytes, n, word_starts, 0, opts, &t);
    if (rc != GBPE_OK) return rc;
    std::vector<uint32_t> batch((size_t)t->batch * 4);
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t total = 0;
    bool stopped = false;
    while (total < t->needed && !stopped) {
        uint32_t done = 0, es = 0;
        rc = gbpe_trainer_step(t, t->batch, batch.data(), &done, &es);
        if (rc != GBPE_OK) break;
        for (uint32_t i = 0; i < done; ++i) {
            if (merges_out && total + i < merges_cap) memcpy(merges_out + 4 * (total + i), &batch[4 * i], 16);
        }
        total += done;
        stopped = es != 0;
        if (cb) {
            gbpe_progress p{};
            p.merge_index = total;
            p.total_merges = t->needed;
            p.best_count = done ? batch[4 * (done - 1) + 3] : 0u;
            p.symbol_count = t->n;
            p.batch_merges = done;
            p.early_stop = stopped;
            p.elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (cb(&p, batch.data(), user) != 0) {
                rc = gbpe_set_error(ctx, GBPE_E_CANCELLED, "training cancelled by progress callback");
                break;
            }
        }
        if (done == 0 && !stopped) break;
    }
    if (n_merges) *n_merges = total < merges_cap || !merges_out ? total : merges_cap;
    if (early_stop) *early_stop = stopped ? 1u : 0u;
    if (rc == GBPE_OK && merges_out && total > merges_cap)
        rc = gbpe_set_error(ctx, GBPE_E_CAPACITY, "merges_out too small: need %u", total);
    gbpe_trainer_destroy(t);
    return rc;
}

extern "C" int gbpe_word_boundary(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, uint8_t* ws_out) {
    if (!ctx || (!bytes && n) || (!ws_out && n)) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    if (n == 0) return GBPE_OK;
    hipStream_t s = ctx->stream;
    uint8_t* d = nullptr;
    GBPE_HIP(ctx, pool_malloc(ctx, &d, 2 * n));
    hipError_t e = hipMemcpyAsync(d, bytes, n, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_symbols<uint32_t>, dim3((uint32_t)gbpe_div_up(n, TPB)), dim3(TPB), 0, s, d,
                       (const uint8_t*)nullptr, (uint32_t*)nullptr, n, d + n);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(ws_out, d + n, n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    pool_free(ctx, d);
    if (e != hipSuccess) return gbpe_set_error(ctx, GBPE_E_DEVICE, "word boundary failed: %s", hipGetErrorString(e));
    return GBPE_OK;
}

