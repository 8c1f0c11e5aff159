// Context, errors and device-memory helpers of the gpubpe C-ABI.
// Replaces the reference's WebGPU device bring-up (engine.js:143-177,
// engine.js:216-238): one HIP device + one stream per context.

#include "common.h"

#include <cstdarg>

int gbpe_set_error(gbpe_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

// Kernel inventory (engine.js:234 logs the pipeline count).  Each entry maps
// one of this library's kernels to the reference kernel(s) it replaces.
static const char* const kKernelNames[] = {
    "k_symbols",         // bpe_word_boundary (train.wgsl:144) + byte widening (trainer.js:49)
    "k_count_full",      // bpe_clear_table + bpe_pair_count_b (train.wgsl:188, 366): initial / rebuild count
    "k_select",          // bpe_find_max_pair_final_det + bpe_setup_merge (train.wgsl:276, 329)
    "k_delta",           // bpe_merge_reduce_b (train.wgsl:433) + incremental pair-count deltas
    "k_compact",         // bpe_prefix_sum_scan_blocks_* + bpe_finalize_compact_b (train.wgsl:522-731) + stale-tail pairs
    "k_refresh",         // bpe_find_max_pair4 (train.wgsl:204) on touched blocks + symbol_count update
    "k_trie_walk",       // trie_tokenizer_chunked (tokenize.wgsl:88): k_trie_walk_v5 (packed double array) / nested form
    "k_chunk_scan",      // trie_prefix_sum (tokenize.wgsl:199)
    "k_chunk_compact",   // trie_tokenizer_compact (tokenize.wgsl:225): k_chunk_compact4
    "k_pretok",          // PreTokenizer GPT-4 word starts (pre_tokenizer.mjs:226-292): k_pt_scan1/2 + k_pt_mark
    "k_me_walk",         // TokenizerManager.encode (tokenizer-manager.js:13-61): per-segment rank-order BPE
    "k_me_compact",      // its token compaction
};

// ── context memory pool (common.h GbpePool) ───────────────────────────────
static uint64_t pool_class(uint64_t b) {
    if (b < 256) return 256;
    uint64_t p2 = 256;
    while (p2 < b) p2 <<= 1;
    if (p2 <= (64u << 10)) return p2;
    const uint64_t step = p2 >> 4;   // p2 < 2b: a step below b / 8, so <= 1/8 slack above 64 KiB
    return (b + step - 1) / step * step;
}

static void pool_release(GbpePool& pl, bool host, uint64_t keep) {
    while (pl.idle_bytes > keep && !pl.idle.empty()) {
        auto it = std::prev(pl.idle.end());   // largest first
        if (host) hipHostFree(it->second);
        else hipFree(it->second);
        pl.idle_bytes -= it->first;
        pl.idle.erase(it);
    }
}

// GBPE_DEBUG poison=1: every pool block handed out is filled with 0xA5 first (tests:
// no trainer buffer may rely on a fresh allocation's contents)
static void pool_poison(gbpe_ctx* ctx, void* p, uint64_t cls, bool host) {
    static const bool on = gbpe_debug_knob("poison", 0) != 0;
    if (!on) return;
    if (host) memset(p, 0xA5, cls);
    else (void)hipMemsetAsync(p, 0xA5, cls, ctx->stream);
}

hipError_t gbpe_pool_alloc(gbpe_ctx* ctx, void** p, uint64_t bytes, bool host) {
    *p = nullptr;
    const uint64_t cls = pool_class(bytes ? bytes : 1);
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    GbpePool& pl = host ? ctx->hpool : ctx->dpool;
    auto it = pl.idle.lower_bound(cls);
    if (it != pl.idle.end() && it->first <= cls + cls / 8) {   // (a reused block holds <= 1/8 more than its class)
        *p = it->second;
        pl.busy[*p] = it->first;
        pl.idle_bytes -= it->first;
        pl.idle.erase(it);
        ++pl.hits;
        pool_poison(ctx, *p, pl.busy[*p], host);
        return hipSuccess;
    }
    ++pl.misses;
    hipError_t e = host ? hipHostMalloc(p, cls, hipHostMallocDefault) : hipMalloc(p, cls);
    if (e != hipSuccess) {   // idle blocks back to the device, then once more
        (void)hipGetLastError();
        pool_release(pl, host, 0);
        e = host ? hipHostMalloc(p, cls, hipHostMallocDefault) : hipMalloc(p, cls);
    }
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    pl.busy[*p] = cls;
    pool_poison(ctx, *p, cls, host);
    return hipSuccess;
}

void gbpe_pool_free(gbpe_ctx* ctx, void* p, bool host) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    GbpePool& pl = host ? ctx->hpool : ctx->dpool;
    auto it = pl.busy.find(p);
    if (it == pl.busy.end()) {   // (not a pool block)
        if (host) hipHostFree(p);
        else hipFree(p);
        return;
    }
    pl.idle.emplace(it->second, p);
    pl.idle_bytes += it->second;
    pl.busy.erase(it);
    pool_release(pl, host, host ? (1ull << 30) : ctx->total_mem / 2);
}

void gbpe_pool_trim(gbpe_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    pool_release(ctx->dpool, false, 0);
    pool_release(ctx->hpool, true, 0);
}

// device memory outside the pool (encode, pre-tokenizer and merge-encode buffers):
// a failed hipMalloc gives the pool's idle blocks back and tries once more, so a
// context that trained first can still encode
hipError_t gbpe_dev_malloc(gbpe_ctx* ctx, void** p, uint64_t bytes) {
    hipError_t e = hipMalloc(p, bytes ? bytes : 1);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        gbpe_pool_trim(ctx);
        e = hipMalloc(p, bytes ? bytes : 1);
    }
    return e;
}

extern "C" {

const char* gbpe_version(void) { return "gpubpe 0.6 (gfx950, abi 5)"; }

int gbpe_abi_version(void) { return GBPE_ABI_VERSION; }

uint64_t gbpe_trainer_stats_size(void) { return sizeof(gbpe_trainer_stats); }

int gbpe_kernel_count(void) { return (int)(sizeof(kKernelNames) / sizeof(kKernelNames[0])); }

const char* gbpe_kernel_name(int i) {
    if (i < 0 || i >= gbpe_kernel_count()) return nullptr;
    return kKernelNames[i];
}

int gbpe_ctx_create(int device_ordinal, gbpe_ctx** out) {
    if (!out) return GBPE_E_INVALID;
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) return GBPE_E_DEVICE;
    if (device_ordinal < 0 || device_ordinal >= count) return GBPE_E_INVALID;
    auto* ctx = new (std::nothrow) gbpe_ctx();
    if (!ctx) return GBPE_E_OOM;
    ctx->device = device_ordinal;
    if (hipSetDevice(device_ordinal) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return GBPE_E_DEVICE;
    }
    ctx->own_stream = ctx->stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device_ordinal) == hipSuccess) {
        ctx->total_mem = prop.totalGlobalMem;
        ctx->num_cu = prop.multiProcessorCount;
    }
    for (auto& ev : ctx->ev) hipEventCreate(&ev);
    if (hipHostMalloc((void**)&ctx->enc_host_total, 16, hipHostMallocDefault) != hipSuccess) {
        hipStreamDestroy(ctx->stream);
        delete ctx;
        return GBPE_E_OOM;
    }
    *out = ctx;
    return GBPE_OK;
}

void gbpe_ctx_destroy(gbpe_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    hipFree(ctx->enc_scratch);
    hipFree(ctx->enc_counts);
    hipFree(ctx->enc_in);
    hipFree(ctx->enc_out);
    hipFree(ctx->pt_agg);
    if (ctx->enc_host_total) hipHostFree(ctx->enc_host_total);
    gbpe_pool_trim(ctx);   // (blocks still busy belong to trainers the caller did not destroy)
    for (auto& ev : ctx->ev)
        if (ev) hipEventDestroy(ev);
    if (ctx->copy_stream) {
        hipStreamSynchronize(ctx->copy_stream);
        hipStreamDestroy(ctx->copy_stream);
    }
    if (ctx->own_stream) {
        hipStreamSynchronize(ctx->own_stream);
        hipStreamDestroy(ctx->own_stream);
    }
    delete ctx;
}

int gbpe_ctx_set_stream(gbpe_ctx* ctx, void* stream) {
    if (!ctx) return GBPE_E_INVALID;
    GBPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->stream = (hipStream_t)stream;   // taken literally: NULL is the device's null stream
    return GBPE_OK;
}

void* gbpe_ctx_get_stream(gbpe_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int gbpe_ctx_limits(gbpe_ctx* ctx, uint64_t* max_buffer_size) {
    if (!ctx || !max_buffer_size) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *max_buffer_size = ctx->total_mem;
    return GBPE_OK;
}

const char* gbpe_last_error(const gbpe_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int gbpe_ctx_trim(gbpe_ctx* ctx) {
    if (!ctx) return GBPE_E_INVALID;
    gbpe_pool_trim(ctx);
    return GBPE_OK;
}

int gbpe_device_alloc(gbpe_ctx* ctx, uint64_t bytes, void** dptr) {
    if (!ctx || !dptr) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess) {   // the pool's idle blocks first
        (void)hipGetLastError();
        gbpe_pool_trim(ctx);
        GBPE_HIP(ctx, hipMalloc(dptr, bytes ? bytes : 1));
    }
    return GBPE_OK;
}

int gbpe_device_free(gbpe_ctx* ctx, void* dptr) {
    if (!ctx) return GBPE_E_INVALID;
    GBPE_HIP(ctx, hipFree(dptr));
    return GBPE_OK;
}

int gbpe_memcpy_h2d(gbpe_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    if (!ctx) return GBPE_E_INVALID;
    GBPE_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    GBPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return GBPE_OK;
}

int gbpe_memcpy_d2h(gbpe_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    if (!ctx) return GBPE_E_INVALID;
    GBPE_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    GBPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return GBPE_OK;
}

int gbpe_synchronize(gbpe_ctx* ctx) {
    if (!ctx) return GBPE_E_INVALID;
    GBPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return GBPE_OK;
}

}  // extern "C"
