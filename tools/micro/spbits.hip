// Micro-benchmark of the sector filter build (train.hip k_sp_bits) on a
// synthetic u16 body: 256-symbol sectors, Zipf-like tokens over a 32K vocab,
// a word start every ~5 symbols.  Variants:
//   loads   read the sectors only
//   sig     pair signatures in LDS (the trainer's signature-only rebuild)
//   sig+bits  plus the token bitmap (rows = token, W words per row)
//   colbits   bitmap built by one workgroup per 32-sector column: an LDS
//             token -> mask table, then plain stores of whole words
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <cmath>
#include <random>

constexpr int TPB = 256;
constexpr uint32_t SIGW = 32;
constexpr uint32_t WS = 0x8000u, TM = 0x7FFFu;

__device__ __forceinline__ uint32_t fmix(uint32_t x) {
    x = (x ^ (x >> 16)) * 0x7feb352du;
    x = (x ^ (x >> 15)) * 0x846ca68bu;
    return x ^ (x >> 16);
}
__device__ __forceinline__ void sig_set(uint32_t* sig, uint32_t pid) {
    const uint32_t h = fmix(pid ^ 0x9E3779B9u), b1 = h & 1023u, b2 = (h >> 16) & 1023u;
    const uint32_t m1 = 1u << (b1 & 31u), m2 = 1u << (b2 & 31u);
    if (!(sig[b1 >> 5] & m1)) atomicOr(&sig[b1 >> 5], m1);
    if (!(sig[b2 >> 5] & m2)) atomicOr(&sig[b2 >> 5], m2);
}

template <int MODE>
__global__ __launch_bounds__(TPB) void k_bits(const uint16_t* __restrict__ body, const uint2* __restrict__ sec,
                                              uint32_t nk, uint32_t* __restrict__ bits, uint32_t W,
                                              uint32_t* __restrict__ sig) {
    __shared__ uint32_t ssig[TPB / 64][SIGW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x * (TPB / 64) + wid;
    const bool live = k < nk;
    if (lane < (int)SIGW) ssig[wid][lane] = 0u;
    __syncthreads();
    uint32_t acc = 0;
    if (live) {
        const uint2 e = sec[k];
        const uint32_t bit = 1u << (k & 31u);
        uint32_t* col = MODE == 2 ? bits + (k >> 5) : nullptr;
        for (uint32_t j = lane; j < e.y; j += 64) {
            const uint32_t x = body[e.x + j];
            const uint32_t tok = x & TM;
            acc += x;
            if (MODE == 2) {
                uint32_t* wp = col + (uint64_t)tok * W;
                if (!(*wp & bit)) atomicOr(wp, bit);
            }
            if (MODE >= 1 && j && !(x & WS)) {
                const uint32_t tp = body[e.x + j - 1] & TM;
                if (tp && tok) sig_set(ssig[wid], (tp << 16) | tok);
            }
        }
    }
    __syncthreads();
    if (MODE >= 1 && live && lane < (int)SIGW) sig[(uint64_t)k * SIGW + lane] = ssig[wid][lane];
    if (MODE == 0 && acc == 0x12345u) sig[k] = acc;
}

// one workgroup per bitmap column (32 sectors): LDS open-addressing table token -> mask
constexpr int CT = 4096;
__global__ __launch_bounds__(TPB) void k_colbits(const uint16_t* __restrict__ body, const uint2* __restrict__ sec,
                                                 uint32_t nk, uint32_t* __restrict__ bits, uint32_t W) {
    __shared__ uint32_t key[CT], msk[CT];
    for (int i = threadIdx.x; i < CT; i += TPB) { key[i] = 0xFFFFFFFFu; msk[i] = 0u; }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t c = blockIdx.x;
    for (uint32_t s = wid; s < 32; s += TPB / 64) {
        const uint32_t k = c * 32 + s;
        if (k >= nk) break;
        const uint2 e = sec[k];
        for (uint32_t j = lane; j < e.y; j += 64) {
            const uint32_t tok = body[e.x + j] & TM;
            uint32_t h = fmix(tok) & (CT - 1);
            for (int p = 0; p < 64; ++p) {
                const uint32_t o = atomicCAS(&key[h], 0xFFFFFFFFu, tok);
                if (o == 0xFFFFFFFFu || o == tok) { atomicOr(&msk[h], 1u << s); break; }
                h = (h + 1) & (CT - 1);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < CT; i += TPB)
        if (key[i] != 0xFFFFFFFFu) bits[(uint64_t)key[i] * W + c] = msk[i];
}

int main(int argc, char** argv) {
    const uint32_t nsec = argc > 1 ? atoi(argv[1]) : 236000, V = 32768, SW = 256;
    const uint64_t n = (uint64_t)nsec * SW;
    std::vector<uint16_t> h(n);
    std::mt19937 rng(7);
    std::vector<double> cdf(V);
    double z = 0;
    for (uint32_t i = 1; i < V; ++i) cdf[i] = (z += 1.0 / i);
    std::uniform_real_distribution<double> U(0, z);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t t = (uint32_t)(std::lower_bound(cdf.begin() + 1, cdf.end(), U(rng)) - cdf.begin());
        h[i] = (uint16_t)(t | (rng() % 5 == 0 ? WS : 0));
    }
    std::vector<uint2> hs(nsec);
    for (uint32_t k = 0; k < nsec; ++k) hs[k] = make_uint2(k * SW, SW - (k % 7));
    const uint32_t W = (nsec + 31) / 32;
    uint16_t* body; uint2* sec; uint32_t *bits, *sig;
    hipMalloc(&body, n * 2 + 256);
    hipMalloc(&sec, nsec * 8);
    hipMalloc(&bits, (uint64_t)V * W * 4);
    hipMalloc(&sig, (uint64_t)nsec * SIGW * 4);
    hipMemcpy(body, h.data(), n * 2, hipMemcpyHostToDevice);
    hipMemcpy(sec, hs.data(), nsec * 8, hipMemcpyHostToDevice);
    printf("nsec %u, body %.1f MB, bitmap %.1f MB\n", nsec, n * 2 / 1e6, (double)V * W * 4 / 1e6);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 g((nsec + 3) / 4);
    const char* names[] = {"loads", "sig", "sig+bits", "memset bits", "colbits", "memset+colbits"};
    for (int v = 0; v < 6; ++v) {
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            switch (v) {
            case 0: hipLaunchKernelGGL(k_bits<0>, g, dim3(TPB), 0, 0, body, sec, nsec, bits, W, sig); break;
            case 1: hipLaunchKernelGGL(k_bits<1>, g, dim3(TPB), 0, 0, body, sec, nsec, bits, W, sig); break;
            case 2:
                hipMemsetAsync(bits, 0, (uint64_t)V * W * 4, 0);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_bits<2>, g, dim3(TPB), 0, 0, body, sec, nsec, bits, W, sig);
                break;
            case 3: hipMemsetAsync(bits, 0, (uint64_t)V * W * 4, 0); break;
            case 4:
                hipMemsetAsync(bits, 0, (uint64_t)V * W * 4, 0);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_colbits, dim3(W), dim3(TPB), 0, 0, body, sec, nsec, bits, W);
                break;
            case 5:
                hipMemsetAsync(bits, 0, (uint64_t)V * W * 4, 0);
                hipLaunchKernelGGL(k_colbits, dim3(W), dim3(TPB), 0, 0, body, sec, nsec, bits, W);
                break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("%-16s %9.1f us  %7.1f GB/s of body\n", names[v], best * 1e3, n * 2 / (best * 1e-3) / 1e9);
    }
    // check colbits == sig+bits bitmap
    std::vector<uint32_t> b1((uint64_t)V * W), b2((uint64_t)V * W);
    hipMemsetAsync(bits, 0, (uint64_t)V * W * 4, 0);
    hipLaunchKernelGGL(k_bits<2>, g, dim3(TPB), 0, 0, body, sec, nsec, bits, W, sig);
    hipMemcpy(b1.data(), bits, b1.size() * 4, hipMemcpyDeviceToHost);
    hipMemsetAsync(bits, 0, (uint64_t)V * W * 4, 0);
    hipLaunchKernelGGL(k_colbits, dim3(W), dim3(TPB), 0, 0, body, sec, nsec, bits, W);
    hipMemcpy(b2.data(), bits, b2.size() * 4, hipMemcpyDeviceToHost);
    printf("colbits %s\n", b1 == b2 ? "equal" : "DIFFERENT");
    return 0;
}
