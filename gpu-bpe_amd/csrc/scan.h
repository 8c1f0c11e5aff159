// Two-level exclusive scan of per-chunk u32 counts (chunk-level parallel
// encode outputs): k_chunk_scan1 per 4096 counts, k_chunk_scan2 over the block
// totals.  Replaces the single-thread trie_prefix_sum (tokenize.wgsl:199-208).
#pragma once
#include "common.h"

namespace {

constexpr int SCAN_TPB = 1024;
constexpr int SCAN_PER = 4;                       // counts per thread in k_chunk_scan1
constexpr int SCAN_BLK = SCAN_TPB * SCAN_PER;     // 4096 chunks per scan block

// per 4096-chunk block: local exclusive prefix (in place) + block total
__global__ __launch_bounds__(SCAN_TPB) void k_chunk_scan1(const uint32_t* __restrict__ counts, uint64_t nchunks,
                                                          uint32_t* __restrict__ local, uint64_t* __restrict__ blocksum) {
    __shared__ uint32_t wsum[SCAN_TPB / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_BLK + (uint64_t)threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        v[k] = (base + k < nchunks) ? counts[base + k] : 0u;
        s += v[k];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t run = incl - s;
    for (int w = 0; w < wid; ++w) run += wsum[w];
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        if (base + k < nchunks) local[base + k] = run;
        run += v[k];
    }
    if (threadIdx.x == SCAN_TPB - 1) blocksum[blockIdx.x] = run;
}

// exclusive scan of block totals (one workgroup); writes the grand total
__global__ __launch_bounds__(SCAN_TPB) void k_chunk_scan2(uint64_t* __restrict__ blocksum, uint64_t nblk,
                                                          uint64_t* __restrict__ total) {
    __shared__ uint64_t wsum[SCAN_TPB / 64];
    const uint64_t per = (nblk + SCAN_TPB - 1) / SCAN_TPB;
    const uint64_t lo = threadIdx.x * per, hi = min(lo + per, nblk);
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += blocksum[i];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
        uint64_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint64_t run = incl - s;
    for (int w = 0; w < wid; ++w) run += wsum[w];
    for (uint64_t i = lo; i < hi; ++i) {
        uint64_t v = blocksum[i];
        blocksum[i] = run;
        run += v;
    }
    if (threadIdx.x == SCAN_TPB - 1) *total = run;
}

// one wave per chunk: coalesced copy of its tokens to the final offset
}  // namespace
