// Micro-benchmark: read bandwidth of a 8192-symbol (16 KB) tile per workgroup
// with (A) 64 contiguous bytes per lane (4 x dwordx4 at lane stride 64 B) versus
// (B) coalesced vectors (lane stride 16 B, 1 KiB per wave-instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_lane_contig(const uint4* __restrict__ in, uint32_t* out) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;   // in uint4
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = in[base + k];
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) x ^= v[k].x + v[k].y + v[k].z + v[k].w;
    if (x == 0x12345678u) out[blockIdx.x] = x;
}

__global__ __launch_bounds__(256) void k_coalesced(const uint4* __restrict__ in, uint32_t* out) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + wid * 256 + lane;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = in[base + k * 64];
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) x ^= v[k].x + v[k].y + v[k].z + v[k].w;
    if (x == 0x12345678u) out[blockIdx.x] = x;
}

int main() {
    const uint64_t tiles = 4100, bytes = tiles * 16384;
    uint4* in;
    uint32_t* out;
    hipMalloc(&in, bytes + 4096);
    hipMalloc(&out, tiles * 4);
    hipMemset(in, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int pass = 0; pass < 2; ++pass) {
        for (int kind = 0; kind < 2; ++kind) {
            const int reps = 200;
            hipEventRecord(e0);
            for (int r = 0; r < reps; ++r) {
                if (kind == 0) hipLaunchKernelGGL(k_lane_contig, dim3(tiles), dim3(256), 0, 0, in, out);
                else hipLaunchKernelGGL(k_coalesced, dim3(tiles), dim3(256), 0, 0, in, out);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (pass) printf("%s: %.2f us/launch, %.0f GB/s\n", kind ? "coalesced" : "lane_contig", 1e3 * ms / reps,
                             bytes / (ms / reps * 1e-3) / 1e9);
        }
    }
    return 0;
}
