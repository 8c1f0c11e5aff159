// Internal definitions shared by the gpubpe HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gpubpe.h"

// Memory pool of a context (the header's "the library owns and pools device
// memory"; the reference pools its GPU buffers, tokenizer.js:30-46, 108-166):
// the buffers a trainer or shard frees go back to the pool and the next one of the
// context takes them (the same stream orders every use), so creating and
// destroying a trainer costs no hipMalloc / hipFree once the pool is warm.  Sizes
// round up to classes of <= 1/8 slack; a miss allocates; an allocation that finds
// no memory frees the idle blocks and tries again (so do the library's allocations
// outside the pool, gbpe_dev_malloc); idle blocks above half the device's memory are
// freed at once, and gbpe_ctx_trim gives every idle block back (for allocators
// outside the library).
struct GbpePool {
    std::multimap<uint64_t, void*> idle;          // class bytes -> block
    std::unordered_map<void*, uint64_t> busy;     // block -> class bytes
    uint64_t idle_bytes = 0, hits = 0, misses = 0;
};

struct gbpe_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;   // created by gbpe_ctx_create; `stream` may be a caller's
    hipStream_t copy_stream = nullptr;  // gbpe_encode's device-to-host copies of finished slices (created on first use)
    uint64_t total_mem = 0;
    int num_cu = 0;
    std::string err;
    // encode pool (tokenizer.js:30-46 buffer pool: grows, never shrinks)
    void* enc_scratch = nullptr;  uint64_t enc_scratch_bytes = 0;
    void* enc_counts = nullptr;   uint64_t enc_counts_bytes = 0;
    void* enc_in = nullptr;       uint64_t enc_in_bytes = 0;
    void* enc_out = nullptr;      uint64_t enc_out_bytes = 0;
    uint32_t* enc_host_total = nullptr;   // pinned
    void* pt_agg = nullptr;       uint64_t pt_agg_bytes = 0;   // pre-tokenizer block aggregates
    hipEvent_t ev[8] = {};
    double enc_ms[3] = {0, 0, 0};
    GbpePool dpool, hpool;   // device / pinned host blocks of trainers and shards
    std::mutex pool_mu;
};

// pooled allocations (api.hip); host = pinned host memory (hipHostMalloc)
hipError_t gbpe_pool_alloc(gbpe_ctx* ctx, void** p, uint64_t bytes, bool host = false);
void gbpe_pool_free(gbpe_ctx* ctx, void* p, bool host = false);
void gbpe_pool_trim(gbpe_ctx* ctx);
hipError_t gbpe_dev_malloc(gbpe_ctx* ctx, void** p, uint64_t bytes);   // hipMalloc, trimming the pool on OOM
template <typename T>
inline hipError_t dev_malloc(gbpe_ctx* c, T** p, uint64_t n) { return gbpe_dev_malloc(c, (void**)p, n); }
template <typename T>
inline hipError_t pool_malloc(gbpe_ctx* c, T** p, uint64_t n) { return gbpe_pool_alloc(c, (void**)p, n); }
inline void pool_free(gbpe_ctx* c, void* p) { gbpe_pool_free(c, p); }
template <typename T>
inline hipError_t pool_hmalloc(gbpe_ctx* c, T** p, uint64_t n) { return gbpe_pool_alloc(c, (void**)p, n, true); }
inline void pool_hfree(gbpe_ctx* c, void* p) { gbpe_pool_free(c, p, true); }

// ── error helpers ──────────────────────────────────────────────────────────
int gbpe_set_error(gbpe_ctx* ctx, int code, const char* fmt, ...);

#define GBPE_HIP(ctx, call)                                                              \
    do {                                                                                 \
        hipError_t _e = (call);                                                          \
        if (_e != hipSuccess)                                                            \
            return gbpe_set_error((ctx), _e == hipErrorOutOfMemory ? GBPE_E_OOM           \
                                                                   : GBPE_E_DEVICE,      \
                                  "%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), \
                                  __FILE__, __LINE__);                                   \
    } while (0)

#define GBPE_LAUNCH_CHECK(ctx) GBPE_HIP(ctx, hipGetLastError())

// runs `f` when the scope ends (device buffers of a call freed on every return path)
template <typename F>
struct GbpeScopeExit {
    F f;
    ~GbpeScopeExit() { f(); }
};
template <typename F>
GbpeScopeExit<F> gbpe_scope_exit(F f) { return GbpeScopeExit<F>{f}; }

// ── device helpers ─────────────────────────────────────────────────────────
__device__ __forceinline__ uint32_t gbpe_fmix32(uint32_t x) {
    // Murmur3 finaliser — the reference's pair hash (train.wgsl:62-67)
    x = (x ^ (x >> 16)) * 0x7feb352du;
    x = (x ^ (x >> 15)) * 0x846ca68bu;
    return x ^ (x >> 16);
}

__host__ __device__ static inline uint64_t gbpe_div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// Debug / test overrides: GBPE_DEBUG="key=value,key=value" (DESIGN §6 lists the
// keys); every other tuning value is a compiled default
inline long gbpe_debug_knob(const char* key, long def) {
    const char* e = getenv("GBPE_DEBUG");
    if (!e) return def;
    const size_t kl = strlen(key);
    for (const char* p = e; *p;) {
        if (!strncmp(p, key, kl) && p[kl] == '=') return strtol(p + kl + 1, nullptr, 10);
        const char* c = strchr(p, ',');
        if (!c) break;
        p = c + 1;
    }
    return def;
}

// GPT-4 rule word starts of device bytes on ctx->stream (pretok.hip)
int gbpe_pretok_gpt4_launch(gbpe_ctx* ctx, const uint8_t* d_bytes, uint64_t n, uint8_t* d_ws);
