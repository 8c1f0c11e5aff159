// Internal definitions shared by the gpubpe HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpubpe.h"

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
};

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
