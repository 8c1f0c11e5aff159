// Residency probe (diagnostic): how many 256-thread workgroups with L bytes of
// static LDS and ~R live VGPRs per lane run at once on this GPU.  1024
// workgroups each stay ~20 us; the resident set is the number that started
// before the first one finished.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/lds_resid.hip -o tools/micro/lds_resid && tools/micro/lds_resid
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int L, int R>
__global__ __launch_bounds__(256) void k_probe(unsigned long long* out, int spin_ticks, const unsigned* src) {
    __shared__ unsigned int buf[L / 4];
    const unsigned long long t0 = wall_clock64();
    unsigned v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) v[k] = src[(threadIdx.x + 256 * k) & 4095];
    for (int i = threadIdx.x; i < L / 4; i += 256) buf[i] = i;
    __syncthreads();
    while (wall_clock64() - t0 < (unsigned long long)spin_ticks) {
        __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = v[k] * 3u + (unsigned)k;   // keeps every register live
    }
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) s ^= v[k];
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t0 + (buf[(blockIdx.x * 7) % (L / 4)] & 0u);
        out[2 * blockIdx.x + 1] = t1 + (s == 0x12345678u ? 1u : 0u);
    }
}

template <int L, int R>
void run(unsigned long long* d, const unsigned* src, int nwg) {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, (const void*)k_probe<L, R>);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((k_probe<L, R>), dim3(nwg), dim3(256), 0, 0, d, 2000, src);
        (void)hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(2 * nwg);
    (void)hipMemcpy(h.data(), d, 2 * nwg * 8, hipMemcpyDeviceToHost);
    unsigned long long first_end = ~0ull;
    for (int i = 0; i < nwg; ++i) first_end = std::min(first_end, h[2 * i + 1]);
    int res = 0;
    for (int i = 0; i < nwg; ++i) res += h[2 * i] < first_end;
    printf("LDS %6d B, %3d VGPRs: %4d of %d resident (%.2f per CU)\n", L, fa.numRegs, res, nwg, res / 256.0);
}

int main() {
    unsigned long long* d = nullptr;
    unsigned* src = nullptr;
    const int nwg = 1024;
    (void)hipMalloc(&d, 2 * nwg * 8);
    (void)hipMalloc(&src, 4096 * 4);
    (void)hipMemset(src, 1, 4096 * 4);
    run<4096, 8>(d, src, nwg);
    run<33360, 8>(d, src, nwg);
    run<50032, 8>(d, src, nwg);
    run<4096, 96>(d, src, nwg);
    run<33360, 96>(d, src, nwg);
    run<4096, 120>(d, src, nwg);
    run<33360, 120>(d, src, nwg);
    run<4096, 200>(d, src, nwg);
    (void)hipFree(d);
    (void)hipFree(src);
    return 0;
}
