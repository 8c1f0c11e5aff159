// FETCH_SIZE / WRITE_SIZE calibration on the access patterns of k_body, k_refresh
// and the trie walk (MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated only for
// 16-B/lane streaming reads, where it reports half the bytes).  Every kernel
// touches a known set of DISTINCT 128-B lines of a 2 GiB buffer (no line is read
// twice inside a kernel, and each kernel has its own region, so nothing is
// served by a cache another kernel warmed), so the counter can be divided by
// the bytes the kernel requests and by the lines it touches:
//   stream16     16 B per lane, coalesced (the guide's calibrated case)
//   gather4      one 4-B load per lane, every lane on its own line
//                (bitmap words, table keys, signature words)
//   gather8      one 8-B load per lane, own line (sector extents, block maxima)
//   gather16     one 16-B load per lane, own line
//   wave256      each wave reads 256 contiguous bytes (4 B per lane) at a random
//                256-B aligned place (a sector of ~128 u16 symbols)
//   wave2k       each wave reads 2 KB contiguous (2 x 16 B per lane: one
//                256-slot k_refresh block)
//   store4       one 4-B store per lane, own line (scattered rewrites)
//   store256     each wave writes 256 contiguous bytes (a rewritten sector)
//   atomic4      one no-return 4-B atomicAdd per lane, own line (table flush)
// Run:  rocprofv3 --pmc FETCH_SIZE -- ./fetch_cal   and  --pmc WRITE_SIZE;
// tools/fetch_cal.py joins the counters with the byte counts printed here.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int TPB = 256;
constexpr uint64_t LINE = 128;

// the i-th distinct line of a region of `nl` lines (nl a power of two, P odd):
// a permutation, so lines are distinct and scattered
__device__ __forceinline__ uint64_t line_of(uint64_t i, uint64_t nl) { return (i * 0x9E3779B1ull) & (nl - 1); }

__global__ __launch_bounds__(TPB) void k_stream16(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * TPB) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <typename T>
__global__ __launch_bounds__(TPB) void k_gather(const uint8_t* __restrict__ base, uint64_t nl, uint64_t n,
                                                uint32_t* __restrict__ out) {
    const uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
    if (i >= n) return;
    const T v = *reinterpret_cast<const T*>(base + line_of(i, nl) * LINE + 16);
    uint32_t acc;
    if constexpr (sizeof(T) == 16) acc = v.x ^ v.y ^ v.z ^ v.w;
    else if constexpr (sizeof(T) == 8) acc = v.x ^ v.y;
    else acc = v;
    if (acc == 0x12345678u) out[0] = acc;
}

// one wave per segment of SEG bytes at a scattered, SEG-aligned place
template <int SEG>
__global__ __launch_bounds__(TPB) void k_wave(const uint8_t* __restrict__ base, uint64_t nseg, uint64_t nw,
                                              uint32_t* __restrict__ out) {
    const uint64_t w = (blockIdx.x * (uint64_t)TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (w >= nw) return;
    const uint8_t* s = base + line_of(w, nseg) * SEG;
    uint32_t acc = 0;
    if constexpr (SEG == 256) {
        acc = reinterpret_cast<const uint32_t*>(s)[lane];
    } else {
        const uint4* q = reinterpret_cast<const uint4*>(s);
#pragma unroll
        for (int k = 0; k < SEG / 1024; ++k) {
            const uint4 v = q[lane + 64 * k];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(TPB) void k_store4(uint8_t* __restrict__ base, uint64_t nl, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
    if (i < n) *reinterpret_cast<uint32_t*>(base + line_of(i, nl) * LINE + 16) = (uint32_t)i;
}

__global__ __launch_bounds__(TPB) void k_store256(uint8_t* __restrict__ base, uint64_t nseg, uint64_t nw) {
    const uint64_t w = (blockIdx.x * (uint64_t)TPB + threadIdx.x) >> 6;
    if (w < nw) reinterpret_cast<uint32_t*>(base + line_of(w, nseg) * 256)[threadIdx.x & 63] = (uint32_t)w;
}

__global__ __launch_bounds__(TPB) void k_atomic4(uint8_t* __restrict__ base, uint64_t nl, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x;
    if (i < n) atomicAdd(reinterpret_cast<uint32_t*>(base + line_of(i, nl) * LINE + 16), 1u);
}

static uint32_t blocks(uint64_t threads) { return (uint32_t)((threads + TPB - 1) / TPB); }

int main() {
    const uint64_t REGION = 256ull << 20;      // per kernel: 256 MiB of distinct lines
    const int NK = 9;
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, REGION * NK));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, REGION * NK));
    CK(hipDeviceSynchronize());
    const uint64_t nl = REGION / LINE;         // 2M lines per region
    const uint64_t n = nl / 2;                 // touch half of them: 1M accesses
    uint8_t* r[NK];
    for (int k = 0; k < NK; ++k) r[k] = buf + REGION * k;
    // a region written by the memset and untouched since: evict it from the
    // on-die caches by streaming 768 MiB of other regions first
    hipLaunchKernelGGL(k_stream16, dim3(2048), dim3(TPB), 0, 0, (const uint4*)(buf + REGION * 6), 3 * REGION / 16, out);
    CK(hipDeviceSynchronize());
    // k_stream16 of region 0 (the guide's case): 256 MiB
    hipLaunchKernelGGL(k_stream16, dim3(2048), dim3(TPB), 0, 0, (const uint4*)r[0], REGION / 16, out);
    printf("{\"kernel\": \"k_stream16\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)REGION,
           (unsigned long long)(REGION / LINE));
    hipLaunchKernelGGL(k_gather<uint32_t>, dim3(blocks(n)), dim3(TPB), 0, 0, r[1], nl, n, out);
    printf("{\"kernel\": \"k_gather<unsigned int>\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(4 * n), (unsigned long long)n);
    hipLaunchKernelGGL(k_gather<uint2>, dim3(blocks(n)), dim3(TPB), 0, 0, r[2], nl, n, out);
    printf("{\"kernel\": \"k_gather<HIP_vector_type<unsigned int, 2u> >\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(8 * n), (unsigned long long)n);
    hipLaunchKernelGGL(k_gather<uint4>, dim3(blocks(n)), dim3(TPB), 0, 0, r[3], nl, n, out);
    printf("{\"kernel\": \"k_gather<HIP_vector_type<unsigned int, 4u> >\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(16 * n), (unsigned long long)n);
    {   // wave256: 1M segments of 256 B (two lines each)
        const uint64_t nseg = REGION / 256, nw = nseg / 2;
        hipLaunchKernelGGL(k_wave<256>, dim3(blocks(nw * 64)), dim3(TPB), 0, 0, r[4], nseg, nw, out);
        printf("{\"kernel\": \"k_wave<256>\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(256 * nw), (unsigned long long)(2 * nw));
    }
    {   // wave2k: 64K segments of 2 KB
        const uint64_t nseg = REGION / 2048, nw = nseg / 2;
        hipLaunchKernelGGL(k_wave<2048>, dim3(blocks(nw * 64)), dim3(TPB), 0, 0, r[5], nseg, nw, out);
        printf("{\"kernel\": \"k_wave<2048>\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(2048 * nw), (unsigned long long)(16 * nw));
    }
    CK(hipDeviceSynchronize());
    // writes (regions 6-8 were streamed above: they are re-dirtied here, WRITE_SIZE counts write-backs)
    hipLaunchKernelGGL(k_store4, dim3(blocks(n)), dim3(TPB), 0, 0, r[6], nl, n);
    printf("{\"kernel\": \"k_store4\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(4 * n), (unsigned long long)n);
    {
        const uint64_t nseg = REGION / 256, nw = nseg / 2;
        hipLaunchKernelGGL(k_store256, dim3(blocks(nw * 64)), dim3(TPB), 0, 0, r[7], nseg, nw);
        printf("{\"kernel\": \"k_store256\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(256 * nw), (unsigned long long)(2 * nw));
    }
    hipLaunchKernelGGL(k_atomic4, dim3(blocks(n)), dim3(TPB), 0, 0, r[8], nl, n);
    printf("{\"kernel\": \"k_atomic4\", \"requested\": %llu, \"lines\": %llu}\n", (unsigned long long)(4 * n), (unsigned long long)n);
    CK(hipDeviceSynchronize());
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
