// Micro-benchmark: cost of a dependent kernel boundary versus an in-kernel grid
// barrier on MI355X.  Each "step" every workgroup reads a word the previous
// step wrote (from another workgroup) and writes its own.
//   launch   one kernel per step, back to back on one stream
//   coop     one cooperative kernel, a cooperative-groups grid.sync() per step
//   atomic   one cooperative kernel, a hand-rolled sense-reversing barrier
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
#include <cstdlib>

namespace cg = cooperative_groups;

__global__ void k_step(uint32_t* buf, uint32_t nwg, uint32_t it) {
    if (threadIdx.x == 0) {
        const uint32_t src = (blockIdx.x + 1) % nwg;
        const uint32_t v = __hip_atomic_load(&buf[src * 64 + (it & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        buf[blockIdx.x * 64 + ((it + 1) & 1)] = v + 1;
    }
}

__global__ void k_coop(uint32_t* buf, uint32_t nwg, uint32_t iters) {
    cg::grid_group g = cg::this_grid();
    for (uint32_t it = 0; it < iters; ++it) {
        if (threadIdx.x == 0) {
            const uint32_t src = (blockIdx.x + 1) % nwg;
            const uint32_t v = __hip_atomic_load(&buf[src * 64 + (it & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            buf[blockIdx.x * 64 + ((it + 1) & 1)] = v + 1;
        }
        g.sync();
    }
}

__global__ void k_atomic(uint32_t* buf, uint32_t nwg, uint32_t iters, uint32_t* bar) {
    for (uint32_t it = 0; it < iters; ++it) {
        if (threadIdx.x == 0) {
            const uint32_t src = (blockIdx.x + 1) % nwg;
            const uint32_t v = __hip_atomic_load(&buf[src * 64 + (it & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&buf[blockIdx.x * 64 + ((it + 1) & 1)], v + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // arrive: release this workgroup's writes, then count in; the last one
            // bumps the generation
            const uint32_t gen = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t n = __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (n == nwg - 1) {
                __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&bar[1], gen + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                uint32_t spins = 0;
                while (__hip_atomic_load(&bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 26)) break;   // never hang the box
                }
            }
        }
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const uint32_t nwg = argc > 1 ? atoi(argv[1]) : 463, iters = 2000;
    uint32_t *buf, *bar;
    hipMalloc(&buf, nwg * 256);
    hipMalloc(&bar, 256);
    hipMemset(buf, 0, nwg * 256);
    hipMemset(bar, 0, 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev = 0, coop = 0, maxb = 0;
    hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&maxb, (const void*)k_coop, 256, 0);
    printf("nwg %u, cooperative %d, coop blocks/CU %d\n", nwg, coop, maxb);
    for (int pass = 0; pass < 2; ++pass) {
        float ms;
        hipEventRecord(e0);
        for (uint32_t it = 0; it < iters; ++it) hipLaunchKernelGGL(k_step, dim3(nwg), dim3(256), 0, 0, buf, nwg, it);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (pass) printf("launch  %.2f us/step\n", 1e3 * ms / iters);
        uint32_t n = nwg, it2 = iters;
        void* args[] = {&buf, &n, &it2};
        hipEventRecord(e0);
        hipError_t e = hipLaunchCooperativeKernel((const void*)k_coop, dim3(nwg), dim3(256), args, 0, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (pass) printf("coop    %.2f us/step (%s)\n", 1e3 * ms / iters, hipGetErrorString(e));
        void* args2[] = {&buf, &n, &it2, &bar};
        hipEventRecord(e0);
        e = hipLaunchCooperativeKernel((const void*)k_atomic, dim3(nwg), dim3(256), args2, 0, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (pass) printf("atomic  %.2f us/step (%s)\n", 1e3 * ms / iters, hipGetErrorString(e));
    }
    return 0;
}
