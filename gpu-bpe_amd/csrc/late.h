// Late-merge loop: ONE 1024-thread workgroup runs a whole step's
// sector-sparse merges back to back.
//
// Late in training a merge has a few hundred sites: the two-launch form
// (k_body + k_refresh, §2b) spends ~18 us per merge on launch boundaries and
// dependent round trips through the pair table, not on bytes.  k_late keeps
// what every merge touches in its own LDS:
//   * the ZONE (the stream's dense tail, where the reference's compaction quirk
//     acts: train.wgsl:605-607 + 698/727) and its stale ping-pong buffer, both
//     resident for the whole launch — the zone pass is LDS work only;
//   * a HOT SET: the pairs whose count exceeded a threshold tau at the launch
//     (exact counts), plus every pair a merge creates with a count > tau.  The
//     argmax (count, then smallest a<<16|b: train.wgsl:83-85, 276-318) is taken
//     over the hot set.  Every pair outside it had a count <= tau at the launch
//     and can only have gained since through deltas the loop saw: W sums, per
//     merge, the largest positive delta any pair outside the set received, so
//     every outside count is <= tau + W.  A hot-set maximum > tau + W is
//     therefore the table maximum; otherwise the launch ends before that merge
//     and the host refreshes the set (the launch never guesses).
// The body sectors (the word lexicon's store, §2c) stay in HBM: per merge one
// load of the two bitmap rows, one of the candidates' extents and signatures,
// one of the sectors.  Count deltas go to the hot set and to a log that
// k_late_apply adds to the global pair table after the launch (the table is
// exact again at every step boundary: k_refresh re-maxes it, the next step's
// refresh reads it).
#pragma once

#include "train_dev.h"

namespace {

constexpr int LATE_BT = 1024;          // 16 waves (512 threads: no spills, but slower per merge: DESIGN §2d)
constexpr uint32_t LATE_HS = 2048;     // hot-set slots (LDS hash: pid -> exact count), two per thread
constexpr uint32_t LATE_K = 1024;      // most pairs a refresh puts in the hot set
constexpr uint32_t LATE_HP = 32;       // hot-set probes
constexpr int LATE_LT = 4096;          // per-merge LDS delta table
constexpr uint32_t LATE_CAP = LATE_BT; // candidate sectors per pass (one per thread)
constexpr uint32_t LATE_NB = 8192;     // count histogram bins of the refresh
constexpr uint32_t LATE_WW = 4;        // bitmap words per thread and pass
constexpr uint32_t LATE_FC = 2;        // candidates per thread the fast body path filters during the zone pass
template <typename S>
struct LateDim {
    static constexpr int ZPT = (sizeof(S) == 2 ? 16 : 8) * 1024 / LATE_BT;   // zone positions per thread
    static constexpr uint32_t ZCAP = (uint32_t)LATE_BT * ZPT;    // 16K u16 / 8K u32 symbols (32 KB)
    static_assert(ZPT <= 32, "thread masks are 32 bits");
    static constexpr uint32_t ZV = ZCAP * sizeof(S) / 16;        // 16-byte vectors per buffer
    static constexpr uint32_t WB = ZCAP / 8 * 3;                 // window staging: mc <= z / 3 < 3/8 ZCAP
};

constexpr uint32_t LATE_KB = 512;      // most table blocks the refresh gathers from (k_hot_sel)
constexpr uint32_t LATE_BL = 1024;     // block list capacity (those plus any dirty block)

// the hot-set refresh between launches (k_hot_sel + k_hot_gather_blocks; the
// full-table k_hot_hist + k_hot_gather are the reference form)
struct LateHot {
    uint32_t ticket, tau, nhot, ok;
    uint32_t nblist;
    uint32_t pad[11];
    uint32_t hist[LATE_NB];
    uint2 list[LATE_K];
    uint32_t blist[LATE_BL];
};

// tau from the table's block maxima (exact at a step boundary: k_refresh has
// re-maxed every dirty block; a block still flagged dirty is listed anyway):
// the smallest threshold with at most LATE_KB blocks whose maximum exceeds it.
// Every pair above tau sits in one of those blocks, so gathering them is
// complete; more than LATE_K such pairs leave the set unusable (the step runs
// with k_body).  One workgroup: 4,096 block maxima at 1 GiB instead of the whole
// table (two 8 MB passes and ~10^5 contended histogram atomics per launch).
__global__ __launch_bounds__(1024) void k_hot_sel(Table tb, LateHot* __restrict__ h) {
    __shared__ uint32_t sh[LATE_NB];
    __shared__ uint32_t s_red[16], s_min[16], s_n, s_tau;
    const uint32_t t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6;
    for (uint32_t i = t; i < LATE_NB; i += 1024) sh[i] = 0u;
    if (t == 0) s_n = 0u;
    __syncthreads();
    for (uint32_t b = t; b < tb.nblk; b += 1024) {
        const uint32_t c = tb.dirty[b] ? LATE_NB - 1 : (uint32_t)(tb.bmax[b] >> 32);
        if (c) atomicAdd(&sh[c < LATE_NB - 1 ? c : LATE_NB - 1], 1u);
    }
    __syncthreads();
    constexpr uint32_t PER = LATE_NB / 1024;
    uint32_t v[PER], tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        v[j] = sh[t * PER + j];
        tot += v[j];
    }
    // blocks above this thread's bins: the wave's inclusive scan from the top, then the waves above
    const uint32_t incl_up = wave_sum_u32(tot) - wave_scan_incl_u32(tot) + tot;   // lanes >= this one
    if (lane == 0) s_red[wid] = incl_up;
    __syncthreads();
    uint32_t above = incl_up - tot;
    for (int w2 = wid + 1; w2 < 16; ++w2) above += s_red[w2];
    uint32_t run = above, cmin = 0xFFFFFFFFu;
#pragma unroll
    for (int j = PER - 1; j >= 0; --j) {
        run += v[j];
        const uint32_t c = t * PER + (uint32_t)j;
        if (c >= 1u && run <= LATE_KB) cmin = c;
    }
    cmin = wave_min_u32(cmin);
    if (lane == 0) s_min[wid] = cmin;
    __syncthreads();
    if (t == 0) {
        uint32_t c = s_min[0];
        for (int w2 = 1; w2 < 16; ++w2) c = min(c, s_min[w2]);
        s_tau = c != 0xFFFFFFFFu ? c - 1u : 0xFFFFFFFFu;
    }
    __syncthreads();
    const uint32_t tau = s_tau;
    if (tau != 0xFFFFFFFFu)
        for (uint32_t b = t; b < tb.nblk; b += 1024)
            if (tb.dirty[b] || (uint32_t)(tb.bmax[b] >> 32) > tau) {
                const uint32_t i = atomicAdd(&s_n, 1u);
                if (i < LATE_BL) h->blist[i] = b;
            }
    __syncthreads();
    if (t == 0) {
        h->tau = tau;
        h->ok = tau != 0xFFFFFFFFu && s_n <= LATE_BL ? 1u : 0u;
        h->nblist = s_n < LATE_BL ? s_n : LATE_BL;
        h->nhot = 0u;
    }
}

// every pair above tau of the listed blocks into the hot list (one slot per thread)
__global__ __launch_bounds__(256) void k_hot_gather_blocks(Table tb, LateHot* __restrict__ h) {
    if (!h->ok) return;
    const uint32_t tau = h->tau, nb = h->nblist;
    for (uint32_t j = blockIdx.x; j < nb; j += gridDim.x) {
        const uint64_t slot = ((uint64_t)h->blist[j] << BLK_LOG2) + threadIdx.x;
        const uint2 e = tb.slots[slot];
        if (e.x && (int32_t)e.y > (int32_t)tau) {
            const uint32_t p = atomicAdd(&h->nhot, 1u);
            if (p < LATE_K) h->list[p] = e;
        }
    }
}

// Count histogram of the live pairs (bins clamped at LATE_NB - 1); the last
// workgroup picks tau: the smallest threshold with at most LATE_K pairs above
// it (ok = 0 when even the top bin holds more), then zeroes the histogram.
__global__ __launch_bounds__(256) void k_hot_hist(Table tb, LateHot* __restrict__ h) {
    __shared__ uint32_t sh[LATE_NB];
    __shared__ uint32_t s_last, s_red[4], s_min[4];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < LATE_NB; i += 256) sh[i] = 0u;
    __syncthreads();
    const uint64_t nq = ((uint64_t)tb.mask + 1) / 2;   // two slots per 16-byte load
    const uint4* q = reinterpret_cast<const uint4*>(tb.slots);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + t; i < nq; i += (uint64_t)gridDim.x * 256) {
        const uint4 e = q[i];
        if (e.x && (int32_t)e.y > 0) atomicAdd(&sh[e.y < LATE_NB - 1 ? e.y : LATE_NB - 1], 1u);
        if (e.z && (int32_t)e.w > 0) atomicAdd(&sh[e.w < LATE_NB - 1 ? e.w : LATE_NB - 1], 1u);
    }
    __syncthreads();
    for (uint32_t i = t; i < LATE_NB; i += 256)
        if (sh[i]) atomicAdd(&h->hist[i], sh[i]);
    __threadfence();
    __syncthreads();
    if (t == 0) s_last = atomicAdd(&h->ticket, 1u) == gridDim.x - 1u ? 1u : 0u;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    // S(c) = pairs with count >= c (bin NB-1: counts >= NB-1).  Pairs above tau =
    // S(tau + 1); the smallest c >= 1 with S(c) <= K gives tau = c - 1.
    constexpr uint32_t PER = LATE_NB / 256;
    uint32_t v[PER], tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        v[j] = __hip_atomic_load(&h->hist[t * PER + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tot += v[j];
    }
    // exclusive suffix over threads (threads above this one)
    const int lane = t & 63, wid = t >> 6;
    uint32_t incl = tot;   // inclusive suffix within the wave (lanes >= this one)
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_down(incl, off);
        if (lane + off < 64) incl += o;
    }
    if (lane == 0) s_red[wid] = incl;
    __syncthreads();
    uint32_t above = incl - tot;   // this wave's lanes above
    for (int w2 = wid + 1; w2 < 4; ++w2) above += s_red[w2];
    uint32_t run = above, cmin = 0xFFFFFFFFu;
#pragma unroll
    for (int j = PER - 1; j >= 0; --j) {
        run += v[j];
        const uint32_t c = t * PER + (uint32_t)j;
        if (c >= 1u && run <= LATE_K) cmin = c;
    }
    for (int off = 32; off > 0; off >>= 1) cmin = min(cmin, (uint32_t)__shfl_xor(cmin, off));
    if (lane == 0) s_min[wid] = cmin;
    __syncthreads();
    if (t == 0) {
        uint32_t c = s_min[0];
        for (int w2 = 1; w2 < 4; ++w2) c = min(c, s_min[w2]);
        h->ok = c != 0xFFFFFFFFu ? 1u : 0u;
        h->tau = c != 0xFFFFFFFFu ? c - 1u : 0xFFFFFFFFu;
        h->nhot = 0u;
        h->ticket = 0u;
    }
    for (uint32_t i = t; i < LATE_NB; i += 256) h->hist[i] = 0u;
}

// every live pair with a count > tau into the hot list (at most LATE_K of them)
__global__ __launch_bounds__(256) void k_hot_gather(Table tb, LateHot* __restrict__ h) {
    const uint32_t tau = h->tau;
    if (!h->ok) return;
    const uint64_t nq = ((uint64_t)tb.mask + 1) / 2;
    const uint4* q = reinterpret_cast<const uint4*>(tb.slots);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * 256) {
        const uint4 e = q[i];
        const bool k0 = e.x && (int32_t)e.y > (int32_t)tau, k1 = e.z && (int32_t)e.w > (int32_t)tau;
        const uint32_t c = (k0 ? 1u : 0u) + (k1 ? 1u : 0u);
        if (!c) continue;
        uint32_t p = atomicAdd(&h->nhot, c);
        if (k0 && p < LATE_K) h->list[p++] = make_uint2(e.x, e.y);
        if (k1 && p < LATE_K) h->list[p] = make_uint2(e.z, e.w);
    }
}

// a late merge's count deltas that found no room in the LDS table: straight to
// the log (the hot set misses them, so the launch ends after this merge)
struct LateSpill {
    uint2* log;
    uint32_t cap;
    uint32_t* pos;    // LDS: next log entry
    uint32_t* inval;  // LDS: the hot set is no longer complete
    uint32_t* ltn;    // LDS: slots of the delta table this merge touched
};
__device__ void table_add(const LateSpill& sp, DevState* st, uint32_t pid, uint32_t d) {
    const uint32_t i = atomicAdd(sp.pos, 1u);
    if (i < sp.cap) sp.log[i] = make_uint2(pid, d);
    else atomicOr(&st->err, ERR_TABLE_FULL);
    *sp.inval = 1u;
}

// the per-merge delta table: LdsTab's probing, plus the list of slots a merge
// filled, so the walk reads those instead of scanning every slot
struct LateTab {
    uint32_t key[LATE_LT];
    uint32_t val[LATE_LT];
    uint16_t list[LATE_LT];
};
__device__ __forceinline__ void lds_add(LateTab& t, const LateSpill& sp, DevState* st, uint32_t pid, uint32_t d) {
    const uint32_t h = gbpe_fmix32(pid);
#pragma unroll 1
    for (int p = 0; p < LPROBE; ++p) {
        const uint32_t idx = (h + (uint32_t)((p * (p + 1)) >> 1)) & (LATE_LT - 1);
        const uint32_t k = atomicCAS(&t.key[idx], 0u, pid);
        if (k == 0u) t.list[atomicAdd(sp.ltn, 1u)] = (uint16_t)idx;
        if (k == 0u || k == pid) {
            atomicAdd(&t.val[idx], d);
            return;
        }
    }
    table_add(sp, st, pid, d);
}

__device__ __forceinline__ uint32_t hot_find(const uint32_t* hk, uint32_t pid) {
    const uint32_t h = gbpe_fmix32(pid);
    for (uint32_t p = 0; p < LATE_HP; ++p) {
        const uint32_t s = (h + p) & (LATE_HS - 1);
        const uint32_t k = hk[s];
        if (k == pid) return s;
        if (k == 0u) return 0xFFFFFFFFu;
    }
    return 0xFFFFFFFFu;
}
__device__ __forceinline__ bool hot_insert(uint32_t* hk, uint32_t* hc, uint32_t pid, uint32_t cnt) {
    const uint32_t h = gbpe_fmix32(pid);
    for (uint32_t p = 0; p < LATE_HP; ++p) {
        const uint32_t s = (h + p) & (LATE_HS - 1);
        const uint32_t k = atomicCAS(&hk[s], 0u, pid);
        if (k == 0u) {
            hc[s] = cnt;
            return true;
        }
        if (k == pid) {
            atomicAdd(&hc[s], cnt);
            return true;
        }
    }
    return false;
}

// a wave-uniform value into a scalar register (values read from LDS land in
// vector registers; the loop state is uniform and would hold 2 x 20 of them)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

// phase stamps of a -DGBPE_KTRACE build (tools/ktrace_late.py): every KT_EVERY-th
// merge, slots 0-5 = merge start, selection done, zone reads + candidate filter
// done, zone written + sectors merged, deltas walked, merge closed;
// 6 = candidates << 16 | filtered candidates
#ifdef GBPE_KTRACE
#define LKT(i) do { if (t == 0) kt_put(r, KT_WG - 1u, (i), wall_clock64()); } while (0)
#define LKTV(i, v) do { if (t == 0) kt_put(r, KT_WG - 1u, (i), (v)); } while (0)
#else
#define LKT(i) ((void)0)
#define LKTV(i, v) ((void)0)
#endif

struct LateOut {
    uint2* dlog;            // count deltas of the launch (k_late_apply)
    uint32_t dcap;
    uint32_t* dlog_n;       // entries written
    uint32_t* mlog;         // merge log [a, b, id, count] per round
    uint64_t* bytes;        // bytes moved (body sectors + zone), for the roofline
    uint32_t* stat;         // [0] launches ended by the hot-set bound, [1] ... by a spill / full hot set
};

// per-merge LDS counters, double-buffered by merge parity: merge r's are read
// after its last barrier and zeroed during merge r + 1, so no barrier of their own
enum : int { LC_NPASS = 0, LC_BIG, LC_LTN, LC_WMAX, LC_NCAND, LC_N };

// Per merge, four workgroup barriers:
//   selection  argmax over the hot set                                  | barrier
//   phase 1    zone reads, masks, destroyed pairs (LDS) while the bitmap rows
//              load; then each thread's candidates (<= LATE_FC) load their
//              extents and signatures and the survivors join the sector list | barrier
//   phase 2    zone writes (only where the new zone differs from what the
//              stale buffer already holds: the agreement prefix `eq`), window
//              pairs; one wave per listed sector                      | barrier
//   walk       the merge's touched delta slots -> log, hot set, bound | barrier
// A merge with more candidates (or a bitmap wider than one pass) takes the
// batched body path after its zone writes.
template <typename S, bool EXACT>
__global__ __launch_bounds__(LATE_BT) void k_late(DevState* st, DevState* zst, S* __restrict__ body,
                                                   uint32_t* __restrict__ lmul, uint2* __restrict__ sec,
                                                   uint32_t* __restrict__ bits, uint32_t W, uint32_t* __restrict__ sig,
                                                   S* __restrict__ zg0, S* __restrict__ zg1, LateHot* __restrict__ hot,
                                                   uint32_t zf, LateOut out) {
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    constexpr int BT = LATE_BT;
    constexpr int ZPT = LateDim<S>::ZPT;
    constexpr uint32_t ZV = LateDim<S>::ZV, WBN = LateDim<S>::WB;
    constexpr int NWAVE = BT / 64;
    constexpr int NW = sizeof(DevState) / 4;
    static_assert(2 * NW <= BT && LC_N * 2 <= BT, "the prologue loads both states in one pass");
    __shared__ uint4 zb[2][ZV];                  // zone and stale buffer (ping-pong)
    __shared__ S wb[WBN];                        // the merge's window source (stale symbols)
    __shared__ uint32_t hk[LATE_HS], hc[LATE_HS];   // hot set
    __shared__ LateTab lt;
    __shared__ uint32_t cs[LATE_CAP];
    __shared__ uint2 ce[LATE_CAP];
    __shared__ union {
        DevState d;
        uint32_t w[NW];
    } g0, z0;
    __shared__ uint64_t s_red[NWAVE];
    __shared__ uint32_t s_sum[NWAVE], s_tl[NWAVE], s_fh[NWAVE], s_rm[NWAVE], s_cs[NWAVE];
    __shared__ uint32_t s_pc[2][LC_N];
    __shared__ uint32_t s_logpos, s_inval, s_gn, s_err;
    __shared__ uint64_t s_bytes, s_tail;
    __shared__ uint32_t s_last[5];   // the last merge's a, b, id, count, window (epilogue only: off the registers)
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;

    // ── prologue: states, zone buffers, hot set ──
    if (t < NW) g0.w[t] = reinterpret_cast<const uint32_t*>(st)[t];
    else if (t < 2 * NW) z0.w[t - NW] = reinterpret_cast<const uint32_t*>(zst)[t - NW];
    for (uint32_t q = t; q < ZV; q += BT) {
        zb[0][q] = reinterpret_cast<const uint4*>(zg0)[q];
        zb[1][q] = reinterpret_cast<const uint4*>(zg1)[q];
    }
    for (uint32_t i = t; i < LATE_HS; i += BT) hk[i] = 0u;
    for (uint32_t i = t; i < (uint32_t)LATE_LT; i += BT) {
        lt.key[i] = 0u;
        lt.val[i] = 0u;
    }
    const uint32_t hok = uni(hot->ok), nhot = uni(hot->nhot), tau = uni(hot->tau);
    if (t < 2 * LC_N) s_pc[t / LC_N][t % LC_N] = 0u;
    if (t == 0) {
        s_logpos = 0u;
        s_inval = 0u;
        s_err = 0u;
        s_bytes = 0ull;
        s_tail = g0.d.tail_total;
        s_last[0] = g0.d.a;
        s_last[1] = g0.d.b;
        s_last[2] = g0.d.nw;
        s_last[3] = g0.d.mc;
        s_last[4] = z0.d.m;
    }
    __syncthreads();
    if (t == 0) hot->nhot = 0u;   // (read above by every thread; the next gather appends from 0)
    const bool usable = hok && nhot <= LATE_K;
    if (usable)
        for (uint32_t i = t; i < nhot; i += BT) {
            const uint2 e = hot->list[i];
            if (!hot_insert(hk, hc, e.x, e.y)) s_inval = 1u;
        }
    __syncthreads();
    // loop state (every thread keeps its own copy: all updates are uniform)
    uint32_t n = uni(g0.d.n), B = uni(g0.d.B), Bp = uni(g0.d.Bp), z = uni(z0.d.n), mc_prev = uni(g0.d.mc_prev);
    uint32_t nid = uni(g0.d.next_id);
    uint64_t Wb = 0;
    uint32_t done = 0, cur = 0, stop = 0, abrt = 0, err = 0;
    uint32_t eq = 0;   // the stale buffer equals the zone on [0, eq)
    const uint32_t budget = uni(g0.d.budget);
    uint32_t ended_by = 0;   // 1: hot-set bound, 2: hot set incomplete
    if (!usable || uni(s_inval) || uni(g0.d.stop) || uni(g0.d.sp_abort) || z > LateDim<S>::ZCAP) ended_by = 2;
    uint64_t bytes = 0;
    for (uint32_t r = 0; ended_by == 0 && r < budget; ++r) {
        const uint32_t par = r & 1u;
        uint32_t* const pc = s_pc[par];
        LKT(0);
        // ── selection over the hot set ──
        uint64_t best = 0;
#pragma unroll
        for (uint32_t j = 0; j < LATE_HS / BT; ++j) {
            const uint32_t i = (uint32_t)t + j * BT;
            const uint32_t k = hk[i], c = hc[i];
            const uint64_t key = ((uint64_t)c << 32) | (uint32_t)~k;
            best = (k && (int32_t)c > 0 && key > best) ? key : best;
        }
        best = wave_max_u64(best);
        if (lane == 0) s_red[wid] = best;
        __syncthreads();
        best = s_red[0];
#pragma unroll
        for (int w2 = 1; w2 < NWAVE; ++w2) best = s_red[w2] > best ? s_red[w2] : best;
        best = uni64(best);
        LKT(1);
        const uint32_t mc = (uint32_t)(best >> 32);
        const uint32_t pid = ~(uint32_t)best;
        const uint32_t a = pid >> 16, b = pid & 0xFFFFu, nw = nid;
        // the bound: every pair outside the set is <= tau + W
        if (best == 0 || (uint64_t)mc <= (uint64_t)tau + Wb) {
            ended_by = 1;
            break;
        }
        if (mc < 2u || nw > 0xFFFFu) {   // train.wgsl:345-348
            stop = 1;
            break;
        }
        if (!EXACT && (uint32_t)(n - Bp) < 2u * mc) {   // (cannot happen, as in sel_inline)
            err |= ERR_SPARSE_WINDOW;
            stop = 1;
            break;
        }
        const uint64_t zneed = std::max<uint64_t>(2ull * mc + mc_prev, (uint64_t)zf * mc) + 2u;
        if (!EXACT && (uint64_t)z < zneed) {   // the zone rule (sel_inline): the host goes dense
            abrt = 1;
            break;
        }
        if (!EXACT && (mc > WBN || (uint32_t)(n - Bp) - mc > LateDim<S>::ZCAP)) {
            ended_by = 2;   // (the zone rule keeps both inside the LDS buffers)
            break;
        }
        const LateSpill spill{out.dlog, out.dcap, &s_logpos, &s_inval, &pc[LC_LTN]};
        // ── commit: log, the merged pair's count to 0 (every occurrence is a site) ──
        if (t == 0) {
            out.mlog[r * 4 + 0] = a;
            out.mlog[r * 4 + 1] = b;
            out.mlog[r * 4 + 2] = nw;
            out.mlog[r * 4 + 3] = mc;
            const uint32_t hi = hot_find(hk, pid);
            if (hi != 0xFFFFFFFFu) hc[hi] -= mc;
            const uint32_t lp = atomicAdd(&s_logpos, 1u);
            if (lp < out.dcap) out.dlog[lp] = make_uint2(pid, 0u - mc);
            else atomicOr(&s_err, ERR_TABLE_FULL);
        }
        if (t < LC_N) s_pc[par ^ 1u][t] = 0u;   // the other parity's counters (read before this merge's first barrier)
        // ── phase 1: the two bitmap rows load while the zone is read ──
        uint32_t bw[LATE_WW];
#pragma unroll
        for (uint32_t q = 0; q < LATE_WW; ++q) {
            const uint32_t w = (uint32_t)t + q * BT;
            bw[q] = w < W ? bits[(uint64_t)a * W + w] & bits[(uint64_t)b * W + w] : 0u;
        }
        S* const C = reinterpret_cast<S*>(zb[cur]);
        S* const P = reinterpret_cast<S*>(zb[cur ^ 1u]);
        const uint32_t lim = EXACT ? z : z - mc;
        const uint32_t i0 = (uint32_t)t * ZPT;
        // this thread's ZPT zone symbols, packed as loaded (positions past z are
        // garbage: every mask below is cut to inb)
        constexpr int XD = ZPT * (int)sizeof(S) / 4;
        uint32_t xq[XD];
#pragma unroll
        for (int q = 0; q < XD / 4; ++q) {
            const uint4 v = zb[cur][t * (XD / 4) + q];
            xq[4 * q] = v.x, xq[4 * q + 1] = v.y, xq[4 * q + 2] = v.z, xq[4 * q + 3] = v.w;
        }
        auto xat = [&](int k) -> uint32_t {
            return sizeof(S) == 2 ? (xq[k >> 1] >> (16 * (k & 1))) & 0xFFFFu : xq[k];
        };
        const uint32_t xm2 = i0 >= 2 ? (uint32_t)C[i0 - 2] : 0u, xm1 = i0 >= 1 ? (uint32_t)C[i0 - 1] : 0u;
        const uint32_t nxr = i0 + ZPT < z ? (uint32_t)C[i0 + ZPT] : 0u;
        uint32_t eb = 0, ea = 0;
#pragma unroll
        for (int k = 0; k < ZPT; ++k) {
            eb |= (xat(k) == b ? 1u : 0u) << k;
            ea |= ((xat(k) & TM) == a ? 1u : 0u) << k;
        }
        const uint32_t inb = lane_mask_n(i0, z, ZPT);
        const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a ? 1u : 0u)) & inb;
        const uint32_t h_m1 = (i0 >= 1 && i0 - 1 < z && xm1 == b && (xm2 & TM) == a) ? 1u : 0u;
        const uint32_t h_nx = (nxr == b && (ea >> (ZPT - 1))) ? 1u : 0u;
        const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_nx << (ZPT + 1));
        const uint32_t below = lane_mask_n(i0, lim, ZPT);
        const uint32_t surv = inb & ~hitm, keep = surv & below;
        const uint32_t rwm = ((hitm >> 1) | (h_nx << (ZPT - 1))) & inb;
        uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
        for (uint32_t i = (lim > 1u ? lim : 1u) + t; i < z; i += BT) {   // stale tail: old pairs destroyed
            const uint32_t xi = C[i];
            if (xi & WS) continue;
            const uint32_t tp = C[i - 1] & TM, ti = xi & TM;
            if (tp && ti && ((tp << 16) | ti) != pid) lds_add(lt, spill, st, (tp << 16) | ti, 0xFFFFFFFFu);
        }
        while (rel) {
            const int k = __ffs(rel) - 1;
            rel &= rel - 1;
            const uint32_t i = i0 + k;
            if (i == 0) continue;
            const uint32_t xi = C[i];
            if (xi & WS) continue;
            const uint32_t xp = C[i - 1];
            const bool hm = (hbits >> k) & 1u, h0 = (hbits >> (k + 1)) & 1u, hp = (hbits >> (k + 2)) & 1u;
            const uint32_t tp = xp & TM, ti = xi & TM;
            if (tp && ti && ((tp << 16) | ti) != pid) lds_add(lt, spill, st, (tp << 16) | ti, 0xFFFFFFFFu);
            if (!h0) {
                if (hm) {
                    const uint32_t t2 = hp ? nw : ti;
                    if (t2) lds_add(lt, spill, st, (nw << 16) | t2, 1u);
                } else if (hp && tp) {
                    lds_add(lt, spill, st, (tp << 16) | nw, 1u);
                }
            }
        }
        // block scan of the kept counts; tail survivors sum to m; the first removed symbol below lim
        const uint32_t kc = __popc(keep);
        const uint32_t incl = wave_scan_incl_u32(kc), tl = wave_sum_u32(__popc(surv & ~below));
        const uint32_t fh = wave_min_u32((hitm & below) ? i0 + (uint32_t)(__ffs(hitm & below) - 1) : 0xFFFFFFFFu);
        if (lane == 63) s_sum[wid] = incl;
        if (lane == 0) {
            s_tl[wid] = tl;
            s_fh[wid] = fh;
        }
        // this thread's candidates (a thread with more, or a wider bitmap: the batched path)
        uint32_t ncnd = 0, c0 = SP_INV, c1 = SP_INV;
#pragma unroll
        for (uint32_t q = 0; q < LATE_WW; ++q) {
            uint32_t c = bw[q];
            const uint32_t w = (uint32_t)t + q * BT;
            while (c) {
                const uint32_t sid = w * 32u + (uint32_t)(__ffs(c) - 1);
                c &= c - 1;
                c0 = ncnd == 0 ? sid : c0;
                c1 = ncnd == 1 ? sid : c1;
                ++ncnd;
            }
        }
        const bool fast = ncnd <= LATE_FC && W <= LATE_WW * (uint32_t)BT;
        uint2 e0 = make_uint2(0u, 0u), e1 = make_uint2(0u, 0u);
        bool k0 = false, k1 = false;
        if (fast && ncnd) {
            e0 = sec[c0];
            k0 = sig_has(sig + (uint64_t)c0 * SP_SIGW, pid);
            if (ncnd > 1) {
                e1 = sec[c1];
                k1 = sig_has(sig + (uint64_t)c1 * SP_SIGW, pid);
            }
            bytes += 16ull * ncnd;
        }
        // the window source (the stale buffer: global n - 2mc of the previous
        // stream), staged before phase 2 rewrites P, while the extents load
        if (!EXACT) {
            const uint32_t src0 = (uint32_t)(n - Bp) - 2u * mc;
            for (uint32_t u = t; u < mc; u += BT) wb[u] = P[src0 + u];
        }
        if (!fast) pc[LC_BIG] = 1u;
        if (ncnd) atomicAdd(&pc[LC_NCAND], ncnd);
        if (k0 || k1) {
            uint32_t q = atomicAdd(&pc[LC_NPASS], (k0 ? 1u : 0u) + (k1 ? 1u : 0u));
            if (k0) {
                if (q < LATE_CAP) {
                    cs[q] = c0;
                    ce[q] = e0;
                }
                ++q;
            }
            if (k1 && q < LATE_CAP) {
                cs[q] = c1;
                ce[q] = e1;
            }
        }
        __syncthreads();   // every read of C and P is done; the sector list is built
        LKT(2);
        uint32_t pre = incl - kc, Kz = 0, m = 0, fhb = 0xFFFFFFFFu;
#pragma unroll
        for (int w2 = 0; w2 < NWAVE; ++w2) {
            pre += w2 < wid ? s_sum[w2] : 0u;
            Kz += s_sum[w2];
            m += s_tl[w2];
            fhb = min(fhb, s_fh[w2]);
        }
        Kz = uni(Kz);
        m = EXACT ? 0u : uni(m);
        const uint32_t npass = uni(pc[LC_NPASS]);
        const bool big = uni(pc[LC_BIG]) != 0u || npass > LATE_CAP;
        // ── phase 2: the new zone into P — kept survivors (A-sides rewritten), then
        //    the window — writing only what P does not already hold; the A-side
        //    rewrites also land in C in place (the next merge's stale source) ──
        uint32_t lastv = 0;
#pragma unroll
        for (int k = 0; k < ZPT; ++k) {
            const bool rw = (rwm >> k) & 1u;
            const uint32_t v = rw ? (nw | (xat(k) & WS)) : xat(k);
            if ((keep >> k) & 1u) {
                const uint32_t d = pre + (uint32_t)__popc(keep & ((1u << k) - 1u));
                if (rw || d >= eq || d != i0 + (uint32_t)k) P[d] = (S)v;
                lastv = v;
            }
            if (rw) C[i0 + k] = (S)v;
        }
        if (!EXACT && m) {
            const uint32_t w0 = mc - m;
            for (uint32_t j = t; j < m; j += BT) {   // the window and its re-added pairs
                const uint32_t x1 = wb[w0 + j];
                P[Kz + j] = (S)x1;
                const uint32_t x0 = j ? (uint32_t)wb[w0 + j - 1] : 0u;
                if (j && !(x1 & WS) && (x0 & TM) && (x1 & TM)) lds_add(lt, spill, st, ((x0 & TM) << 16) | (x1 & TM), 1u);
            }
            if (kc && pre + kc == Kz) {   // the last kept symbol and the window's first
                const uint32_t x1 = wb[w0];
                if (!(x1 & WS) && (lastv & TM) && (x1 & TM)) lds_add(lt, spill, st, ((lastv & TM) << 16) | (x1 & TM), 1u);
            }
        }
        bytes += (t == 0) ? (uint64_t)sizeof(S) * ((uint64_t)z + (EXACT ? 0u : mc) + Kz + m) : 0ull;
        // ── body: one wave per listed sector; the next one's first pass loads
        //    while this one merges ──
        uint32_t removed = 0;
        auto sectors = [&](uint32_t nc) {
            uint32_t nf[5], nfm[4];
            if ((uint32_t)wid < nc)
                sector_first<S>(body + ce[wid].x, lmul ? lmul + ce[wid].x : nullptr, ce[wid].y, nf, nfm);
            for (uint32_t j = wid; j < nc; j += NWAVE) {
                const uint32_t sct = cs[j];
                const uint2 e = ce[j];
                uint32_t cf[5], cfm[4];
#pragma unroll
                for (int k = 0; k < 5; ++k) cf[k] = nf[k];
#pragma unroll
                for (int k = 0; k < 4; ++k) cfm[k] = nfm[k];
                if (j + NWAVE < nc) {
                    const uint2 en = ce[j + NWAVE];
                    sector_first<S>(body + en.x, lmul ? lmul + en.x : nullptr, en.y, nf, nfm);
                }
                uint32_t outc = 0;
#ifdef GBPE_BSPROF
                unsigned long long bsp[6] = {0, 0, 0, 0, 0, 0};
#endif
                const uint32_t rr = body_sector<S, LATE_LT>(body + e.x, lmul ? lmul + e.x : nullptr, e.y, a, b, nw, lt,
                                                             spill, st, sig + (uint64_t)sct * SP_SIGW, outc, cf, cfm,
                                                             nullptr, nullptr, nullptr BSP_PASS);
                if (lane == 0) bytes += (uint64_t)(sizeof(S) + (lmul ? 4u : 0u)) * (e.y + (rr ? outc : 0u));
                if (rr) {
                    removed += rr;
                    if (lane == 0) {
                        sec[sct].y = outc;
                        atomicOr(&bits[(uint64_t)nw * W + (sct >> 5)], 1u << (sct & 31u));
                    }
                }
            }
        };
        [[maybe_unused]] uint32_t nfilt = npass;
        if (!big) {
            sectors(npass);
        } else {
            // batched: every candidate of the bitmap, LATE_CAP at a time, LATE_WW x BT words per pass
            nfilt = 0;
            for (uint32_t wbase = 0;;) {
                uint32_t pcn = 0;
#pragma unroll
                for (uint32_t q = 0; q < LATE_WW; ++q) pcn += __popc(bw[q]);
                const uint32_t cincl = wave_scan_incl_u32(pcn);
                if (lane == 63) s_cs[wid] = cincl;
                __syncthreads();   // (also: the fast list is no longer read)
                uint32_t cpre = cincl - pcn, ncand = 0;
#pragma unroll
                for (int w2 = 0; w2 < NWAVE; ++w2) {
                    cpre += w2 < wid ? s_cs[w2] : 0u;
                    ncand += s_cs[w2];
                }
                ncand = uni(ncand);
                for (uint32_t base = 0; base < ncand; base += LATE_CAP) {
                    {   // this thread's candidates with list positions in [base, base + CAP)
                        uint32_t pos = cpre;
#pragma unroll
                        for (uint32_t q = 0; q < LATE_WW; ++q) {
                            uint32_t c = bw[q];
                            const uint32_t w = wbase + (uint32_t)t + q * BT;
                            while (c) {
                                const int bit = __ffs(c) - 1;
                                c &= c - 1;
                                if (pos >= base && pos < base + LATE_CAP) cs[pos - base] = w * 32u + (uint32_t)bit;
                                ++pos;
                            }
                        }
                    }
                    if (t == 0) s_gn = 0u;
                    __syncthreads();
                    const uint32_t nb = ncand - base < LATE_CAP ? ncand - base : LATE_CAP;
                    uint32_t fs = SP_INV;
                    uint2 fe = make_uint2(0u, 0u);
                    bool fk = false;
                    if ((uint32_t)t < nb) {
                        fs = cs[t];
                        fe = sec[fs];
                        fk = sig_has(sig + (uint64_t)fs * SP_SIGW, pid);
                        bytes += 16ull;
                    }
                    __syncthreads();   // the list is read before it is rewritten
                    if (fk) {
                        const uint32_t qq = atomicAdd(&s_gn, 1u);
                        cs[qq] = fs;
                        ce[qq] = fe;
                    }
                    __syncthreads();
                    const uint32_t nc = uni(s_gn);
                    nfilt += nc;
                    sectors(nc);
                    __syncthreads();   // the list is free for the next batch
                }
                wbase += LATE_WW * BT;
                if (wbase >= W) break;   // (block-uniform)
#pragma unroll
                for (uint32_t q = 0; q < LATE_WW; ++q) {
                    const uint32_t w = wbase + (uint32_t)t + q * BT;
                    bw[q] = w < W ? bits[(uint64_t)a * W + w] & bits[(uint64_t)b * W + w] : 0u;
                }
            }
        }
        if (lane == 0) s_rm[wid] = removed;   // (per lane: body_sector returns the wave's total)
        __syncthreads();   // every delta of the merge is in the table
        LKT(3);
        LKTV(6, ((uint64_t)pc[LC_NCAND] << 16) | nfilt);
        // ── the merge's deltas: log, hot set, bound ──
        const uint32_t nl = uni(pc[LC_LTN]);
        uint32_t wmax = 0;
        for (uint32_t i1 = 0; i1 < nl; i1 += BT) {   // (a uniform trip count: the ballot below)
            const uint32_t i = i1 + (uint32_t)t;
            uint32_t k = 0, d = 0;
            if (i < nl) {
                const uint32_t s = lt.list[i];
                k = lt.key[s];
                d = lt.val[s];
                lt.key[s] = 0u;
                lt.val[s] = 0u;
            }
            const bool live = k && d;
            const unsigned long long bal = __ballot(live);
            uint32_t base = 0;
            if (lane == 0 && bal) base = atomicAdd(&s_logpos, (uint32_t)__popcll(bal));
            base = __builtin_amdgcn_readlane(base, 0);
            if (!live) continue;
            const uint32_t lp = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
            if (lp < out.dcap) out.dlog[lp] = make_uint2(k, d);
            else atomicOr(&s_err, ERR_TABLE_FULL);
            const uint32_t hi = hot_find(hk, k);
            if (hi != 0xFFFFFFFFu) {
                hc[hi] += d;
            } else if ((k >> 16) == nw || (k & 0xFFFFu) == nw) {
                // a pair of the new token: it did not exist before this merge, so d is its count
                if ((int32_t)d > (int32_t)tau && !hot_insert(hk, hc, k, d)) s_inval = 1u;
            } else if ((int32_t)d > 0) {
                wmax = d > wmax ? d : wmax;
            }
        }
        wmax = wave_max_u32(wmax);
        if (lane == 0 && wmax) atomicMax(&pc[LC_WMAX], wmax);
        __syncthreads();   // hot set updated; s_wmax, s_rm, s_inval final
        LKT(4);
        uint32_t body_rm = 0;
#pragma unroll
        for (int w2 = 0; w2 < NWAVE; ++w2) body_rm += s_rm[w2];
        body_rm = uni(body_rm);
        // ── close the merge (k_refresh's finish-2 bookkeeping) ──
        const uint32_t n1 = n - mc, B1 = B - body_rm, z1 = Kz + m;
        if (z1 != n1 - B1) err |= ERR_COUNT_MISMATCH;
        Wb += uni(pc[LC_WMAX]);
        eq = min(uni(fhb), lim);   // the zone just read (now the stale buffer) equals the new one below its first removed symbol
        Bp = B;
        B = B1;
        n = n1;
        z = z1;
        mc_prev = mc;
        if (t == 0) {
            s_tail += m;
            s_last[0] = a;
            s_last[1] = b;
            s_last[2] = nw;
            s_last[3] = mc;
            s_last[4] = m;
        }
        ++nid;
        cur ^= 1u;
        done = r + 1;
        LKT(5);
        if (uni(s_inval)) {
            ended_by = 2;
            break;
        }
    }
    // ── epilogue: zone buffers back, state, counters ──
    __syncthreads();
    for (uint32_t q = t; q < ZV; q += BT) {
        reinterpret_cast<uint4*>(zg0)[q] = zb[0][q];
        reinterpret_cast<uint4*>(zg1)[q] = zb[1][q];
    }
    if (bytes) atomicAdd(&s_bytes, bytes);
    __syncthreads();
    if (t == 0) {
        err |= s_err;
        if (err) atomicOr(&st->err, err);
        st->n = n;
        st->B = B;
        st->Bp = Bp;
        st->body_rm = 0u;
        st->mc_prev = mc_prev;
        st->next_id = nid;
        st->epoch = g0.d.epoch + done;
        st->tail_total = s_tail;
        st->merges_done = done;
        st->sel_round = done;
        st->zlast = z;
        st->a = s_last[0];
        st->b = s_last[1];
        st->nw = s_last[2];
        st->mc = s_last[3];
        st->new_n = n;
        if (stop) st->stop = 1u;
        if (abrt) st->sp_abort = 1u;
        zst->n = z;
        zst->m = s_last[4];
        zst->merges_done = done;
        zst->valid_total = 0u;
        *out.dlog_n = s_logpos < out.dcap ? s_logpos : out.dcap;
        atomicAdd(out.bytes, s_bytes);
        if (ended_by) atomicAdd(&out.stat[ended_by - 1], 1u);
    }
}

// the launch's count deltas into the global table (per-workgroup LDS aggregation)
__global__ __launch_bounds__(256) void k_late_apply(const uint2* __restrict__ dlog, const uint32_t* __restrict__ dlog_n,
                                                    DevState* st, Table tb) {
    __shared__ LdsTab<2048> lt;
    const uint32_t n = *dlog_n;
    const uint32_t per = (uint32_t)gbpe_div_up(n, gridDim.x);
    const uint32_t beg = blockIdx.x * per, end = beg + per < n ? beg + per : n;
    if (beg >= end) return;   // block-uniform
    lds_clear(lt);
    __syncthreads();
    for (uint32_t i = beg + threadIdx.x; i < end; i += 256) {
        const uint2 e = dlog[i];
        lds_add(lt, tb, st, e.x, e.y);
    }
    lds_flush(lt, tb, st);
}

#undef LKT
#undef LKTV

}  // namespace
