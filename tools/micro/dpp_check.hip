// Checks the DPP wave helpers of csrc/train_dev.h (wave_sum_u32, wave_max_u64,
// wave_scan_incl_u32) against plain loops, on the GPU.  Prints FAIL lines.
#include "../../gpu-bpe_amd/csrc/train_dev.h"

#include <cstdio>
#include <vector>

__global__ void k_check(const uint32_t* in, uint32_t* sum, uint64_t* mx, uint32_t* scan) {
    const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const uint32_t v = in[t];
    const uint32_t s = wave_sum_u32(v);
    const uint64_t m = wave_max_u64(((uint64_t)(v % 97u) << 32) | (uint32_t)~(v * 2654435761u));
    const uint32_t c = wave_scan_incl_u32(v & 31u);
    sum[t] = s;
    mx[t] = m;
    scan[t] = c;
}

int main() {
    const int N = 64 * 16;
    std::vector<uint32_t> in(N);
    for (int i = 0; i < N; ++i) in[i] = (uint32_t)(i * 2246822519u + 374761393u) >> 7;
    uint32_t *d_in, *d_sum, *d_scan;
    uint64_t* d_mx;
    (void)hipMalloc(&d_in, N * 4);
    (void)hipMalloc(&d_sum, N * 4);
    (void)hipMalloc(&d_scan, N * 4);
    (void)hipMalloc(&d_mx, N * 8);
    (void)hipMemcpy(d_in, in.data(), N * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(N / 256), dim3(256), 0, 0, d_in, d_sum, d_mx, d_scan);
    std::vector<uint32_t> sum(N), scan(N);
    std::vector<uint64_t> mx(N);
    (void)hipMemcpy(sum.data(), d_sum, N * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(scan.data(), d_scan, N * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(mx.data(), d_mx, N * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int w = 0; w < N / 64; ++w) {
        uint32_t s = 0, c = 0;
        uint64_t m = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t v = in[w * 64 + l];
            s += v;
            const uint64_t k = ((uint64_t)(v % 97u) << 32) | (uint32_t)~(v * 2654435761u);
            m = k > m ? k : m;
        }
        for (int l = 0; l < 64; ++l) {
            const int i = w * 64 + l;
            c += in[i] & 31u;
            if (sum[i] != s && bad++ < 10) printf("FAIL sum wave %d lane %d: %u vs %u\n", w, l, sum[i], s);
            if (mx[i] != m && bad++ < 10) printf("FAIL max wave %d lane %d: %llx vs %llx\n", w, l, (unsigned long long)mx[i], (unsigned long long)m);
            if (scan[i] != c && bad++ < 10) printf("FAIL scan wave %d lane %d: %u vs %u\n", w, l, scan[i], c);
        }
    }
    printf("dpp_check: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 1 : 0;
}
