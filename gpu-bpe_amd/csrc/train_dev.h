// Device side of the training loop (loop state, pair table, LDS tables, the
// dense loop's kernels; the sector-sparse loop is in sparse.h, the word lexicon
// in lexicon.h), shared by the translation units
// train.hip (single-device trainer) and train_lexshard.hip (sharded first
// pass + lexicon hand-over).  Every kernel
// lives in an anonymous namespace: each unit compiles the instances it launches.
#pragma once

#include "common.h"
#include "scan.h"

#include <algorithm>
#include <chrono>
#include <type_traits>
#include <cstdarg>

namespace {

constexpr int TPB = 256;              // threads per block
constexpr int EPT = 32;               // symbols per thread in a tile
constexpr int TILE = TPB * EPT;       // 8192 symbols per tile (16 KiB of u16 in flight per workgroup)
constexpr int LTAB = 2048;            // LDS delta table slots (tail window)
constexpr int LTAB_FULL = 8192;       // LDS table slots for the full recount
constexpr int LPROBE = 24;            // LDS probes before spilling to the global table
constexpr uint32_t BLK_LOG2 = 8;      // 256 table slots per argmax block: one wave re-maxes one (2 x 16 B per lane)
constexpr int SEL_THREADS = 1024;

template <typename S> struct Sym;
template <> struct Sym<uint16_t> { static constexpr uint32_t WS = 0x8000u, TM = 0x7FFFu; };
template <> struct Sym<uint32_t> { static constexpr uint32_t WS = 0x10000u, TM = 0xFFFFu; };

// device-side loop state (the reference's IterState, train.wgsl:45-58)
// Whole-wave reductions and scan on the DPP paths (quad_perm, row mirrors,
// row_shr, row_bcast) plus readlane: no ds_bpermute, which queues behind the
// CU's LDS traffic.  Every lane of the wave must be active (as for __shfl_*).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);   // (readlane is int: no sign extension)
}
// the wave's maximum (uniform)
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    uint64_t o = dpp64<0xB1>(v);   // quad_perm [1,0,3,2]
    v = o > v ? o : v;
    o = dpp64<0x4E>(v);            // quad_perm [2,3,0,1]
    v = o > v ? o : v;
    o = dpp64<0x141>(v);           // row_half_mirror
    v = o > v ? o : v;
    o = dpp64<0x140>(v);           // row_mirror: every lane of a row holds the row's maximum
    v = o > v ? o : v;
    const uint64_t r0 = readlane64(v, 0), r1 = readlane64(v, 16), r2 = readlane64(v, 32), r3 = readlane64(v, 48);
    const uint64_t a = r0 > r1 ? r0 : r1, b = r2 > r3 ? r2 : r3;
    return a > b ? a : b;
}
// Top-2 keys (the paired launch, sparse.h zone_two): every lane holds its own
// first f > second s; keys are unique (one per pair id) except the no-key fills,
// so exactly one lane's f is the wave's first and the second is the largest of
// the other lanes' f and that lane's s (uniform)
__device__ __forceinline__ void wave_top2_u64(uint64_t f, uint64_t s, uint64_t& o1, uint64_t& o2) {
    o1 = wave_max_u64(f);
    o2 = wave_max_u64(f == o1 ? s : f);
}
__device__ __forceinline__ void top2_add(uint64_t& f, uint64_t& s, uint64_t k) {   // (selects: no branches)
    const bool g1 = k > f, g2 = k > s;
    s = g1 ? f : (g2 ? k : s);
    f = g1 ? k : f;
}
__device__ __forceinline__ void top2_merge(uint64_t& f, uint64_t& s, uint64_t g1, uint64_t g2) {
    const uint64_t hi = f > g1 ? f : g1, lo = f > g1 ? g1 : f, s2 = s > g2 ? s : g2;
    f = hi;
    s = lo > s2 ? lo : s2;
}
// the wave's sum (uniform)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += dpp32<0xB1>(v);
    v += dpp32<0x4E>(v);
    v += dpp32<0x141>(v);
    v += dpp32<0x140>(v);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}
// inclusive prefix sum over the wave's lanes
__device__ __forceinline__ uint32_t wave_scan_incl_u32(uint32_t v) {
    v += dpp32<0x111>(v);          // row_shr:1 (lanes shifted in from outside the row add 0)
    v += dpp32<0x112>(v);          // row_shr:2
    v += dpp32<0x114>(v);          // row_shr:4
    v += dpp32<0x118>(v);          // row_shr:8: each row scanned
    v += dpp32<0x142, 0xA>(v);     // row_bcast:15 into rows 1 and 3
    v += dpp32<0x143, 0xC>(v);     // row_bcast:31 into rows 2 and 3
    return v;
}

struct DevState {
    uint32_t n;            // current symbol count
    uint32_t stop;         // early stop (mc < 2 or id > 0xFFFF)
    uint32_t next_id;
    uint32_t a, b, nw;     // merge pair and new id
    uint32_t mc;           // its count
    uint32_t new_n;        // n - mc
    uint32_t m;            // survivors with old index >= new_n (tail window size)
    uint32_t merges_done;  // in this step (reset by the host, trainer.js:239)
    uint32_t used;         // occupied table slots
    uint32_t ndirty;       // dirty-block list length
    uint32_t err;          // error bits
    uint32_t valid_total;  // zone: survivors + 1 (zone_one → k_refresh's layout check)
    uint32_t budget;       // merges allowed in this step
    uint32_t live;         // distinct pairs with count > 0 at the last select
    uint64_t tail_total;   // sum of m
    uint32_t max_live;     // max of `live` over all selects
    uint32_t epoch;        // merge sequence number
    // ── sector-sparse loop (n / new_n above stay GLOBAL; the zone has its own DevState) ──
    uint32_t B;            // body length: symbols in the word-aligned sectors before the zone
    uint32_t Bp;           // body length during the previous merge (stale-window source offset)
    uint32_t body_rm;      // B-sides removed from the body by this merge
    uint32_t sp_abort;     // a selected merge does not fit the zone: not run, host goes dense
    uint32_t sel_round;    // sector-sparse: round + 1 of the merge k_body selected
    uint64_t sp_bytes;     // sector-sparse: bytes moved by the multi-tile zone passes (k_refresh adds them)
    uint32_t zlast;        // sector-sparse: zone length of the rank that holds the zone (global knowledge)
    uint32_t is_last;      // sector-sparse: this rank holds the zone (single GPU: always)
    uint32_t cand;         // candidate sectors of this merge (trace)
    uint32_t hitsec;       // sectors with a site (trace)
    uint32_t mc_prev;      // sector-sparse, single GPU: the last merge's count (k_refresh), for the zone rule
                           // (never written by a commit: a reader beside k_body would see it unchanged)
    uint32_t enter_lim;    // dense loop: end the step at the first merge whose count is <= this (the host
                           // can then enter the sector-sparse loop; 0 = off)
    // ── paired launch (sparse.h zone_two): a second merge in the same k_body ──
    uint32_t mc2;          // the second merge's count (written with the first's commit, used only if acc2)
    uint32_t body_rm2;     // B-sides removed from the body by the second merge
    uint32_t acc2;         // the zone workgroup accepted the second merge (k_refresh consumes and clears it)
    uint32_t paired;       // launches that ran two merges (cumulative)
    uint32_t pair_cand;    // launches whose top two allowed a second merge (cumulative, zone_two)
    uint32_t pair_rej;     // ... that the zone workgroup's window check turned down
};
static_assert(sizeof(DevState) <= 256, "state");

// Offset of a merge's stale-window source in the zone's other buffer: n - 2mc - Bp
// (global positions).  On one device n and Bp are kept modulo 2^32 — a trainer
// built from shards holds more than 2^32 symbols — and only their
// difference, a zone-sized length, is used.
__device__ __forceinline__ uint64_t win_src0(const DevState& g, uint32_t mc) {
    return (uint64_t)(uint32_t)(g.n - g.Bp) - 2ull * mc;
}

// the zone segments' per-merge hand-off (zone_seg; k_refresh zeroes it)
constexpr uint32_t NSEG_MAX = 64;   // one sweeping wave: one lane per segment
constexpr uint32_t ZSEG_SPIN = 1u << 22;
struct ZSegState {
    uint32_t ticket;
    uint32_t pad[15];
    unsigned long long gran[NSEG_MAX][4];   // {1, kept}, {1, tail survivors}, {1, last kept | has kept << 31}
};
constexpr uint32_t ZSEG_WORDS = 16 + NSEG_MAX * 8;   // u32 words k_refresh zeroes (ticket, granules)

// Phase timestamps of the sector-sparse kernels (diagnostic builds only:
// -DGBPE_KTRACE; tools/ktrace.sh).  Every KT_EVERY-th merge, each workgroup
// stores its own wall-clock stamps (plain stores, no shared counters that
// would serialise the launch): k_body workgroups at [m][wg][slot], k_refresh
// workgroups at [m][KT_WG + wg][slot].
#ifdef GBPE_KTRACE
constexpr uint32_t KT_MERGES = 40000, KT_EVERY = 16, KT_WG = 2048, KT_SLOTS = 12;
// __constant__: scalar loads the compiler can hoist, so a stamp is a clock read
// and a store (a __device__ global reloads with a vmcnt wait per stamp, which
// drained the wave's outstanding stores and inflated every phase by ~1 µs)
__constant__ unsigned long long* g_ktr;
__constant__ uint32_t g_kt_base;
__device__ __forceinline__ void kt_put(uint32_t round, uint32_t wg, int i, unsigned long long v) {
    const uint32_t m = g_kt_base + round;
    if (g_ktr && m < KT_MERGES && m % KT_EVERY == 0 && wg < 2 * KT_WG)
        g_ktr[((uint64_t)(m / KT_EVERY) * 2 * KT_WG + wg) * KT_SLOTS + i] = v;
}
#define KT(i) kt_put(round, blockIdx.x, (i), wall_clock64())
#define KTV(i, v) kt_put(round, blockIdx.x, (i), (v))
#define KTR(i) kt_put(round, KT_WG + blockIdx.x, (i), wall_clock64())
// per-wave stamps of the zone workgroup (lane 0 of every wave): rows KT_WG - 8 + wave
#define KTW(i) do { if ((threadIdx.x & 63) == 0) kt_put(round, KT_WG - 8u + (threadIdx.x >> 6), (i), wall_clock64()); } while (0)
#else
#define KTW(i) ((void)0)
#define KT(i) ((void)0)
#define KTV(i, v) ((void)0)
#define KTR(i) ((void)0)
#endif

// Cycle split of body_sector (diagnostic builds only: -DGBPE_BSPROF;
// tools/bsprof.sh): per wave, shader cycles from a pass's start to its hit masks
// (its symbol loads land there), through its count deltas, through its writes;
// the signature flush; passes and sectors.  Summed over every k_body wave of a
// step and printed per step by the host.
#ifdef GBPE_BSPROF
__device__ unsigned long long g_bsprof[8];
#define BSP_ARG , unsigned long long (&bsp)[6]
#define BSP_PASS , bsp
#define BSP_CLK(v) const unsigned long long v = clock64()
#define BSP_ADD(i, x) bsp[i] += (x)
#else
#define BSP_ARG
#define BSP_PASS
#define BSP_CLK(v) ((void)0)
#define BSP_ADD(i, x) ((void)0)
#endif

enum : uint32_t {
    ERR_TABLE_FULL = 1, ERR_COUNT_MISMATCH = 2, ERR_PAIR_MISSING = 4, ERR_SPIN = 8,
    ERR_SPARSE_WINDOW = 128    // sector-sparse: a stale window reaches past the zone's stale buffer
};

struct Table {
    uint2* slots;      // .x = pid (0 = empty), .y = count (u32, wraps for transient negatives)
    uint32_t mask;     // slots - 1
    uint64_t* bmax;    // per block: (count << 32) | ~pid, KEY_NONE when no count is positive
    uint64_t* bmax2;   // per block: the second key (KEY_NONE when fewer than two counts are positive)
    uint32_t* dirty;   // per block flag
    uint32_t* dlist;   // dirty block list
    uint32_t* blive;   // per block: entries with count > 0
    uint32_t nblk;
    uint32_t* used;    // occupied-slot counter (DevState::used or ::dused)
};

// the key of a block without a positive count (count 0, the weakest tie-break)
constexpr uint64_t KEY_NONE = 0xFFFFFFFFull;

// a touched block is re-maxed by the next k_refresh: a plain flag store, nothing waits on it
__device__ __forceinline__ void mark_dirty(const Table& tb, DevState* st, uint32_t slot) {
    (void)st;
    tb.dirty[slot >> BLK_LOG2] = 1u;
}

// global insert-or-add (triangular probing visits every slot of a 2^k table)
__device__ void table_add(const Table& tb, DevState* st, uint32_t pid, uint32_t delta) {
    uint32_t h = gbpe_fmix32(pid) & tb.mask;
    for (uint32_t p = 0; p <= tb.mask; ++p) {
        uint32_t idx = (h + ((p * (p + 1)) >> 1)) & tb.mask;
        uint32_t k = __hip_atomic_load(&tb.slots[idx].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == 0u) {
            k = atomicCAS(&tb.slots[idx].x, 0u, pid);
            if (k == 0u) {
                if (tb.used) __hip_atomic_fetch_add(tb.used, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                k = pid;
            }
        }
        if (k == pid) {
            atomicAdd(&tb.slots[idx].y, delta);
            mark_dirty(tb, st, idx);
            return;
        }
    }
    atomicOr(&st->err, ERR_TABLE_FULL);
}

__device__ uint32_t table_find(const Table& tb, uint32_t pid) {
    uint32_t h = gbpe_fmix32(pid) & tb.mask;
    for (uint32_t p = 0; p <= tb.mask; ++p) {
        uint32_t idx = (h + ((p * (p + 1)) >> 1)) & tb.mask;
        uint32_t k = tb.slots[idx].x;
        if (k == pid) return idx;
        if (k == 0u) return 0xFFFFFFFFu;
    }
    return 0xFFFFFFFFu;
}

// per-workgroup LDS aggregation of (pid, delta)
template <int N>
struct LdsTab {
    uint32_t key[N];
    uint32_t val[N];
    uint32_t ovf;   // an add went straight to the global table (k_tail re-maxes every dirty block then)
};

template <int N>
__device__ __forceinline__ void lds_clear(LdsTab<N>& t) {
    for (int i = threadIdx.x; i < N; i += blockDim.x) { t.key[i] = 0u; t.val[i] = 0u; }
    if (threadIdx.x == 0) t.ovf = 0u;
}

template <int N, typename TB>
__device__ __forceinline__ void lds_add(LdsTab<N>& t, const TB& tb, DevState* st, uint32_t pid, uint32_t d) {
    uint32_t h = gbpe_fmix32(pid);
#pragma unroll 1
    for (int p = 0; p < LPROBE; ++p) {
        uint32_t idx = (h + (uint32_t)((p * (p + 1)) >> 1)) & (N - 1);
        uint32_t k = atomicCAS(&t.key[idx], 0u, pid);
        if (k == 0u || k == pid) {
            atomicAdd(&t.val[idx], d);
            return;
        }
    }
    t.ovf = 1u;
    table_add(tb, st, pid, d);   // LDS table crowded: go straight to the global table
}

// A runtime-sized prefix (a power of two) of an LdsTab: zone_two sizes its table by
// the pair's counts, so a late pair's few hundred deltas do not pay for clearing
// and scanning thousands of slots
struct LdsView {
    uint32_t* key;
    uint32_t* val;
    uint32_t* ovf;
    uint32_t mask;
};
template <int N>
__device__ __forceinline__ LdsView lds_view(LdsTab<N>& t, uint32_t n) {
    return LdsView{t.key, t.val, &t.ovf, n - 1u};
}
__device__ __forceinline__ void lds_clear(LdsView& t) {
    for (uint32_t i = threadIdx.x; i <= t.mask; i += blockDim.x) {
        t.key[i] = 0u;
        t.val[i] = 0u;
    }
    if (threadIdx.x == 0) *t.ovf = 0u;
}
template <typename TB>
__device__ __forceinline__ void lds_add(LdsView& t, const TB& tb, DevState* st, uint32_t pid, uint32_t d) {
    const uint32_t h = gbpe_fmix32(pid);
#pragma unroll 1
    for (int p = 0; p < LPROBE; ++p) {
        const uint32_t idx = (h + (uint32_t)((p * (p + 1)) >> 1)) & t.mask;
        const uint32_t k = atomicCAS(&t.key[idx], 0u, pid);
        if (k == 0u || k == pid) {
            atomicAdd(&t.val[idx], d);
            return;
        }
    }
    *t.ovf = 1u;
    table_add(tb, st, pid, d);   // crowded: straight to the global table
}

// the delta a runtime-sized table holds for pid (0 when absent)
__device__ __forceinline__ uint32_t lds_find(const LdsView& t, uint32_t pid) {
    const uint32_t h = gbpe_fmix32(pid);
#pragma unroll 1
    for (int p = 0; p < LPROBE; ++p) {
        const uint32_t idx = (h + (uint32_t)((p * (p + 1)) >> 1)) & t.mask;
        const uint32_t k = t.key[idx];
        if (k == pid) return t.val[idx];
        if (k == 0u) return 0u;
    }
    return 0u;
}

// K adds of one delta with their home-slot compare-and-swaps issued together: the
// zone passes' stale-tail and window loops were chains of dependent LDS round trips
// (two reads, a CAS, an add per pair, ~4 pairs per thread at late counts); now the
// reads and the CASes of K pairs overlap and the adds need no reply.  A pair whose
// home slot holds another key takes lds_add's full probe.  pid 0 = no pair.
template <int N>
__device__ __forceinline__ uint32_t* tab_key(LdsTab<N>& t) { return t.key; }
template <int N>
__device__ __forceinline__ uint32_t* tab_val(LdsTab<N>& t) { return t.val; }
template <int N>
__device__ __forceinline__ uint32_t tab_mask(const LdsTab<N>&) { return (uint32_t)N - 1u; }
__device__ __forceinline__ uint32_t* tab_key(LdsView& t) { return t.key; }
__device__ __forceinline__ uint32_t* tab_val(LdsView& t) { return t.val; }
__device__ __forceinline__ uint32_t tab_mask(const LdsView& t) { return t.mask; }
template <int K, typename LT, typename TB>
__device__ __forceinline__ void lds_addk(LT& t, const TB& tb, DevState* st, const uint32_t (&kq)[K], uint32_t d) {
    uint32_t* key = tab_key(t);
    uint32_t* val = tab_val(t);
    const uint32_t mask = tab_mask(t);
    uint32_t idx[K], o[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        idx[k] = gbpe_fmix32(kq[k]) & mask;
        o[k] = kq[k] ? atomicCAS(&key[idx[k]], 0u, kq[k]) : 0u;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (!kq[k]) continue;
        if (o[k] == 0u || o[k] == kq[k]) atomicAdd(&val[idx[k]], d);
        else lds_add(t, tb, st, kq[k], d);
    }
}

// Up to 8 (pid, delta) adds with their home-slot key loads issued together: at
// the table's low load factor nearly every live pair sits in its home slot, so
// a batch costs one round trip instead of one per entry; the rest (new keys,
// collisions) take the full probe.  Entries with pid or delta 0 are skipped.
// (Adding at the home slot blind — one returning 64-bit atomic on {pid, count},
// taken back when another pid sits there — measured slower: late 1 GiB merges
// k_body 10.7 -> 11.2 us, code1g 1.42 -> 1.52 s.)
__device__ __forceinline__ void table_add8(const Table& tb, DevState* st, const uint32_t (&kk)[8],
                                           const uint32_t (&vv)[8]) {
    uint32_t hs[8], hk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // (no load for an empty entry: thousands of them hit slot 0's line)
        hs[j] = (kk[j] && vv[j]) ? (gbpe_fmix32(kk[j]) & tb.mask) : 0u;
        hk[j] = (kk[j] && vv[j]) ? __hip_atomic_load(&tb.slots[hs[j]].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (!kk[j] || !vv[j]) continue;
        if (hk[j] == kk[j]) {
            atomicAdd(&tb.slots[hs[j]].y, vv[j]);
            mark_dirty(tb, st, hs[j]);
        } else {
            table_add(tb, st, kk[j], vv[j]);
        }
    }
}

// Flush the workgroup's aggregated deltas into the global table.  Small tables
// (<= 8 slots per thread) are first compacted to a list so every thread does at
// most a few global adds instead of one per slot it owns: a merge's few live
// entries then cost one global round trip, not a serial chain.  Large tables
// (the multi-tile and zone k_delta, the full count) add in batches of 8 per
// thread (table_add8).  The table's contents are consumed (callers clear it
// before reuse).
template <int N, typename TB>
__device__ __forceinline__ void lds_flush(LdsTab<N>& t, const TB& tb, DevState* st) {
    __syncthreads();
    const uint32_t nt = blockDim.x;
    if (N > 8 * (int)nt && N <= 16 * (int)nt && N < 8192) {
        // a large, mostly sparse table (the paired zone pass's 4,096 slots): compacted
        // first, then the live entries added 8 per thread per round trip
        __shared__ uint32_t s_cnt16;
        uint32_t kk[16], vv[16], live = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = threadIdx.x + j * nt;
            kk[j] = i < (uint32_t)N ? t.key[i] : 0u;
            vv[j] = i < (uint32_t)N ? t.val[i] : 0u;
            if (kk[j] && vv[j]) live |= 1u << j;
        }
        if (threadIdx.x == 0) s_cnt16 = 0u;
        __syncthreads();
        uint32_t off = live ? atomicAdd(&s_cnt16, (uint32_t)__popc(live)) : 0u;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if ((live >> j) & 1u) {
                t.key[off] = kk[j];
                t.val[off] = vv[j];
                ++off;
            }
        __syncthreads();
        const uint32_t total = s_cnt16;
        for (uint32_t i0 = threadIdx.x; i0 < total; i0 += 8 * nt) {
            uint32_t k8[8], v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t i = i0 + j * nt;
                k8[j] = i < total ? t.key[i] : 0u;
                v8[j] = i < total ? t.val[i] : 0u;
            }
            table_add8(tb, st, k8, v8);
        }
        return;
    }
    if (N > 8 * (int)nt) {
        for (uint32_t i0 = threadIdx.x; i0 < (uint32_t)N; i0 += 8 * nt) {
            uint32_t kk[8], vv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t i = i0 + j * nt;
                kk[j] = i < (uint32_t)N ? t.key[i] : 0u;
                vv[j] = i < (uint32_t)N ? t.val[i] : 0u;
            }
            table_add8(tb, st, kk, vv);
        }
        return;
    }
    __shared__ uint32_t s_cnt;
    uint32_t kk[8], vv[8], live = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t i = threadIdx.x + j * nt;
        kk[j] = i < (uint32_t)N ? t.key[i] : 0u;
        vv[j] = i < (uint32_t)N ? t.val[i] : 0u;
        if (kk[j] && vv[j]) live |= 1u << j;
    }
    if (threadIdx.x == 0) s_cnt = 0u;
    __syncthreads();
    uint32_t off = live ? atomicAdd(&s_cnt, (uint32_t)__popc(live)) : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if ((live >> j) & 1u) {
            t.key[off] = kk[j];
            t.val[off] = vv[j];
            ++off;
        }
    __syncthreads();
    const uint32_t total = s_cnt;
    for (uint32_t i = threadIdx.x; i < total; i += nt) table_add(tb, st, t.key[i], t.val[i]);
}

// flush of a runtime-sized table (<= 16 slots per thread): the live entries
// compacted, then added 8 per thread per round trip (table_add8)
template <int MAXPER, typename TB>
__device__ __forceinline__ void lds_flush(LdsView& t, const TB& tb, DevState* st) {
    __syncthreads();
    __shared__ uint32_t s_cntv;
    const uint32_t nt = blockDim.x, n = t.mask + 1u;
    uint32_t kk[MAXPER], vv[MAXPER], live = 0;
#pragma unroll
    for (int j = 0; j < MAXPER; ++j) {
        const uint32_t i = threadIdx.x + j * nt;
        kk[j] = i < n ? t.key[i] : 0u;
        vv[j] = i < n ? t.val[i] : 0u;
        if (kk[j] && vv[j]) live |= 1u << j;
    }
    if (threadIdx.x == 0) s_cntv = 0u;
    __syncthreads();
    uint32_t off = live ? atomicAdd(&s_cntv, (uint32_t)__popc(live)) : 0u;
#pragma unroll
    for (int j = 0; j < MAXPER; ++j)
        if ((live >> j) & 1u) {
            t.key[off] = kk[j];
            t.val[off] = vv[j];
            ++off;
        }
    __syncthreads();
    const uint32_t total = s_cntv;
    for (uint32_t i0 = threadIdx.x; i0 < total; i0 += 8 * nt) {
        uint32_t k8[8], v8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t i = i0 + j * nt;
            k8[j] = i < total ? t.key[i] : 0u;
            v8[j] = i < total ? t.val[i] : 0u;
        }
        table_add8(tb, st, k8, v8);
    }
}

template <typename S>
__device__ __forceinline__ void load_tile(const S* __restrict__ cur, uint64_t base, S* __restrict__ tile) {
    // 16 symbols per thread, 16-byte vector loads (buffers are padded to whole tiles)
    constexpr int V = EPT * sizeof(S) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(cur + base) + threadIdx.x * V;
    uint4* dst = reinterpret_cast<uint4*>(tile) + threadIdx.x * V;
#pragma unroll
    for (int v = 0; v < V; ++v) dst[v] = src[v];
}

// ─── kernels ────────────────────────────────────────────────────────────────

// bpe_word_boundary (train.wgsl:111-186) fused with byte→symbol widening
// (trainer.js:49-53) and external-mask tagging (trainer.js:115-121).
__device__ __forceinline__ uint32_t byte_class(uint32_t t) {
    if (t == 0x0Au) return 4u;
    if (t == 0x20u) return 2u;
    if (t - 0x30u <= 9u) return 1u;
    if (t >= 0x80u) return 0u;
    if ((t | 0x20u) - 0x61u <= 25u) return 0u;
    return 3u;
}

template <typename S>
__global__ __launch_bounds__(TPB) void k_symbols(const uint8_t* __restrict__ bytes, const uint8_t* __restrict__ ws_ext,
                                                 S* __restrict__ out, uint64_t n, uint8_t* __restrict__ ws_out) {
    uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    uint32_t tok = bytes[i];
    bool ws;
    if (ws_ext) {
        ws = ws_ext[i] != 0;
    } else if (i == 0) {
        ws = true;
    } else {
        uint32_t c = byte_class(tok), p = byte_class(bytes[i - 1]);
        ws = c != p;
        if (p == 2u && (c == 0u || c == 1u)) ws = false;
        if (c == 2u && p != 2u) ws = true;
        if (p == 4u || c == 4u) ws = true;
    }
    if (out) out[i] = (S)(tok | (ws ? Sym<S>::WS : 0u));
    if (ws_out) ws_out[i] = ws ? 1 : 0;
}

// The same, 16 bytes per thread: one 16-byte load (+ the byte before it), the
// symbols out as whole 16-byte vectors (the byte-per-thread form moved 1 GiB in
// 3.5 ms, its 1- and 2-byte accesses bound by instruction issue).  Needs 16-byte
// aligned bytes and word starts; the output buffer is padded to whole tiles.
template <typename S>
__global__ __launch_bounds__(TPB) void k_symbols_v(const uint8_t* __restrict__ bytes, const uint8_t* __restrict__ ws_ext,
                                                   S* __restrict__ out, uint64_t n) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * TPB + threadIdx.x) * 16u;
    if (i0 >= n) return;
    uint32_t by[16], we[16];
    if (i0 + 16 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(bytes + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) by[k] = (w[k >> 2] >> ((k & 3) * 8)) & 0xFFu;
        if (ws_ext) {
            const uint4 e = *reinterpret_cast<const uint4*>(ws_ext + i0);
            const uint32_t f[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) we[k] = (f[k >> 2] >> ((k & 3) * 8)) & 0xFFu;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            by[k] = i0 + k < n ? bytes[i0 + k] : 0u;
            we[k] = (ws_ext && i0 + k < n) ? ws_ext[i0 + k] : 0u;
        }
    }
    uint32_t prev = i0 ? bytes[i0 - 1] : 0u;
    uint32_t sym[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t tok = by[k];
        bool ws;
        if (ws_ext) {
            ws = we[k] != 0u;
        } else if (i0 + k == 0) {
            ws = true;
        } else {
            const uint32_t c = byte_class(tok), p = byte_class(prev);
            ws = c != p;
            if (p == 2u && (c == 0u || c == 1u)) ws = false;
            if (c == 2u && p != 2u) ws = true;
            if (p == 4u || c == 4u) ws = true;
        }
        sym[k] = tok | (ws ? Sym<S>::WS : 0u);
        prev = tok;
    }
    if (i0 + 16 <= n) {
        if (sizeof(S) == 2) {
            uint4* o = reinterpret_cast<uint4*>(out + i0);
            o[0] = make_uint4(sym[0] | sym[1] << 16, sym[2] | sym[3] << 16, sym[4] | sym[5] << 16, sym[6] | sym[7] << 16);
            o[1] = make_uint4(sym[8] | sym[9] << 16, sym[10] | sym[11] << 16, sym[12] | sym[13] << 16, sym[14] | sym[15] << 16);
        } else {
            uint4* o = reinterpret_cast<uint4*>(out + i0);
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = make_uint4(sym[4 * q], sym[4 * q + 1], sym[4 * q + 2], sym[4 * q + 3]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (i0 + k < n) out[i0 + k] = (S)sym[k];
    }
}

// Full pair count of the current stream into the (cleared) table — once at
// start and on table rebuilds.  Same counting rule as train.wgsl:393-399.
template <typename S>
__global__ __launch_bounds__(TPB) void k_count_full(DevState* st, const S* __restrict__ cur, Table tb) {
    __shared__ LdsTab<LTAB_FULL> lt;
    __shared__ __attribute__((aligned(16))) S tile[TILE];
    __shared__ S prev_last;
    lds_clear(lt);
    const uint32_t n = st->n;
    const uint32_t ntiles = (uint32_t)gbpe_div_up(n, TILE);
    for (uint32_t tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
        const uint64_t base = (uint64_t)tl * TILE;
        __syncthreads();
        load_tile(cur, base, tile);
        if (threadIdx.x == 0) prev_last = base ? cur[base - 1] : (S)0;
        __syncthreads();
#pragma unroll 1
        for (int k = 0; k < EPT; ++k) {
            int li = threadIdx.x * EPT + k;
            uint64_t i = base + li;
            if (i == 0 || i >= n) continue;
            uint32_t x1 = tile[li];
            uint32_t x0 = li ? (uint32_t)tile[li - 1] : (uint32_t)prev_last;
            uint32_t t0 = x0 & Sym<S>::TM, t1 = x1 & Sym<S>::TM;
            if (!(x1 & Sym<S>::WS) && t0 && t1) lds_add(lt, tb, st, (t0 << 16) | t1, 1u);
        }
    }
    lds_flush(lt, tb, st);
}

// The first count, while every symbol is still a byte: only 256 x 256 pairs can
// exist, so each workgroup counts one half of them (first byte < 128 or >= 128)
// in a dense 32K-entry LDS histogram with plain LDS adds — no hashing, no probe —
// over a share of the tiles, and adds its non-zero entries to a dense global
// histogram; k_count_hist then inserts the (<= 65,536) pairs into the table.
// (k_count_full's hashed LDS table took 6.4 ms for 1 GiB of u16 symbols.)
constexpr int CB_T = 1024;
template <typename S>
__global__ __launch_bounds__(CB_T) void k_count_bytes(const S* __restrict__ cur, uint64_t n, uint32_t* __restrict__ gh) {
    __shared__ uint32_t hist[32768];
    for (int i = threadIdx.x; i < 32768; i += CB_T) hist[i] = 0u;
    __syncthreads();
    const uint32_t half = blockIdx.x & 1u, pair = blockIdx.x >> 1, npair = gridDim.x >> 1;
    constexpr int PV = 16 / sizeof(S);   // symbols per 16-byte vector
    const uint64_t nv = gbpe_div_up(n, PV);
    for (uint64_t v = (uint64_t)pair * CB_T + threadIdx.x; v < nv; v += (uint64_t)npair * CB_T) {
        const uint64_t i0 = v * PV;
        uint4 q = *reinterpret_cast<const uint4*>(cur + i0);   // buffers are padded to whole tiles
        const S* e = reinterpret_cast<const S*>(&q);
        uint32_t prev = i0 ? (uint32_t)cur[i0 - 1] : 0u;
#pragma unroll
        for (int k = 0; k < PV; ++k) {
            const uint32_t x = e[k];
            const uint32_t t0 = prev & Sym<S>::TM, t1 = x & Sym<S>::TM;
            if (i0 + k < n && i0 + k > 0 && !(x & Sym<S>::WS) && t0 && t1 && (t0 >> 7) == half)
                atomicAdd(&hist[((t0 & 127u) << 8) | t1], 1u);
            prev = x;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 32768; i += CB_T) {
        const uint32_t c = hist[i];
        if (c) atomicAdd(&gh[(half << 15) | (uint32_t)i], c);
    }
}

__device__ void table_add(const Table& tb, DevState* st, uint32_t pid, uint32_t delta);
__global__ __launch_bounds__(256) void k_count_hist(const uint32_t* __restrict__ gh, DevState* st, Table tb) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;   // (a << 8) | b
    const uint32_t c = gh[i];
    if (c) table_add(tb, st, ((i >> 8) << 16) | (i & 255u), c);
}

__device__ void select_merge(DevState* st, Table tb, uint32_t* __restrict__ log, uint32_t* __restrict__ grpsum,
                             DevState* zst, uint32_t exact);

// (unused launch argument: the selection fused into k_refresh was measured slower)
struct FusedSel {
    uint32_t* log = nullptr;
    uint32_t* grpsum = nullptr;
    uint32_t exact = 0;
};

// recompute block maxima for dirty blocks; with `finish`, also closes the
// merge of `round` (state.symbol_count := new count, train.wgsl:605-607)

template <typename S, bool WIDE = false>
__global__ __launch_bounds__(TPB) void k_refresh(DevState* st, uint32_t round, int finish, Table tb, S* __restrict__ cur,
                                                 const uint32_t* __restrict__ rwlist, DevState* zst,
                                                 uint32_t* __restrict__ clog = nullptr, FusedSel fs = FusedSel(),
                                                 uint64_t* __restrict__ part = nullptr, uint32_t* __restrict__ zseg = nullptr) {
    (void)cur;
    if (zseg && blockIdx.x == 0)   // ZSegState: ticket + granules of the next merge's zone segments
        for (uint32_t i = threadIdx.x; i < ZSEG_WORDS; i += TPB)
            if (i == 0 || i >= 16) zseg[i] = 0u;
    (void)rwlist;
    if (part && finish == 2 && threadIdx.x == 0) KTR(0);
    // this WG's contiguous run of blocks (<= TPB, one per thread): all flags (and,
    // for `part`, the maxima kept from before) in one load — issued first, so
    // block 0's state snapshot below travels in the same round trip instead of
    // before it.  Late steps of a large table take up to 256 blocks per workgroup
    // (the WIDE form: C5's 2^25 slots give 512 partial maxima for the selection to
    // reduce, not 2048; 1,024 blocks per workgroup measured slower, and the narrow
    // form stays a kernel of its own: one body for both cost 1 GiB 1-2 %,
    // profiles/r5/s13)
    __shared__ uint64_t s_dmask[WIDE ? TPB / 64 : 1];
    __shared__ uint64_t s_bm[WIDE ? TPB : 64], s_bm2[WIDE ? TPB : 64];
    const uint32_t per = (tb.nblk + gridDim.x - 1) / gridDim.x;   // <= 64, WIDE: <= TPB (GBPE_LAUNCH_REFRESH)
    constexpr bool wide = WIDE;
    const uint32_t b0 = blockIdx.x * per;
    uint64_t f_bm = 0ull, f_bm2 = 0ull;
    bool f_d = false;
    if (wide || threadIdx.x < 64) {
        const uint32_t blk = b0 + threadIdx.x;
        const bool in = threadIdx.x < per && blk < tb.nblk;
        if (part && in) {
            f_bm = tb.bmax[blk];
            f_bm2 = tb.bmax2[blk];
        }
        f_d = in && tb.dirty[blk];
    }
    // finish == 2: the sector-sparse loop, whose merge was selected inside k_body
    // (sel_inline): the step counters move on here
    // block 0 closes the merge from one snapshot of both states: every field is
    // read (one round trip) before any is written, not one round trip per field
    if (finish && blockIdx.x == 0) {
        constexpr int NW = sizeof(DevState) / 4;
        __shared__ union {
            DevState d;
            uint32_t w[NW];
        } s_g, s_z;
        static_assert(64 + 2 * NW <= TPB, "state snapshot beside the flag loads");
        if (threadIdx.x >= 64 && threadIdx.x < 64 + NW)
            s_g.w[threadIdx.x - 64] = reinterpret_cast<const uint32_t*>(st)[threadIdx.x - 64];
        else if (zst && threadIdx.x >= 64 + NW && threadIdx.x < 64 + 2 * NW)
            s_z.w[threadIdx.x - 64 - NW] = reinterpret_cast<const uint32_t*>(zst)[threadIdx.x - 64 - NW];
        __syncthreads();
        const DevState& g = s_g.d;
        const DevState& z = s_z.d;
        // sector-sparse: the launch's merge index is the state's (a paired launch
        // runs two, so launches and merges part ways)
        const uint32_t r = finish >= 2 ? g.merges_done : round;
        const bool fin = finish >= 2 ? (!g.stop && !g.sp_abort && g.sel_round == r + 1u)
                                     : (!g.stop && g.merges_done == r + 1u);
        if (fin && threadIdx.x == 0) {
            if (zst) {   // sector-sparse: global length, body length, zone length
                const uint32_t k2 = finish >= 2 ? g.acc2 : 0u;   // a second merge ran in this launch
                if (finish >= 2) {
                    st->merges_done = r + 1u + k2;
                    st->next_id = g.next_id + 1u + k2;
                    st->epoch = g.epoch + 1u + k2;
                    st->mc_prev = k2 ? g.mc2 : g.mc;
                    if (k2) {
                        st->acc2 = 0u;
                        st->paired = g.paired + 1u;
                    }
                }
                if (clog) {
                    clog[2 * r] = g.cand;
                    clog[2 * r + 1] = g.hitsec;
                    if (k2) {
                        clog[2 * r + 2] = 0u;
                        clog[2 * r + 3] = 0u;
                    }
                }
                st->cand = 0u;
                st->hitsec = 0u;
                st->tail_total = g.tail_total + z.m;   // (both merges' windows)
                // the second merge ran on the first's stream: its window source lies in the
                // stream whose body was B (not Bp)
                const uint32_t n = g.new_n - (k2 ? g.mc2 : 0u), B = g.B - g.body_rm - g.body_rm2, zn = n - B;
                st->n = n;
                st->Bp = k2 ? g.B - g.body_rm : g.B;
                st->B = B;
                st->body_rm = 0u;
                st->body_rm2 = 0u;
                zst->n = zn;
                st->zlast = zn;
                if (!z.valid_total && g.is_last)   // multi-tile zone: k_delta + k_compact stream it twice, plus the window copy
                    st->sp_bytes = g.sp_bytes + (uint64_t)sizeof(S) * (2ull * z.n + zn + 2ull * g.mc);
                if (z.valid_total && z.valid_total != zn + 1u) atomicOr(&st->err, ERR_COUNT_MISMATCH);
            } else {
                st->tail_total = g.tail_total + g.m;
                st->n = g.new_n;
            }
        }
    }
    // then every wave re-maxes its share of the dirty ones, one 256-slot block at a
    // time (no workgroup barrier per block: a merge dirties a few blocks per
    // workgroup, each holding a few live pairs)
    if (wide || threadIdx.x < 64) {
        if (part) {
            s_bm[threadIdx.x] = f_bm;
            s_bm2[threadIdx.x] = f_bm2;
        }
        const unsigned long long m = __ballot(f_d);
        if ((threadIdx.x & 63) == 0) s_dmask[threadIdx.x >> 6] = m;
    }
    __syncthreads();
    {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        constexpr int NV = (1 << BLK_LOG2) / 2 / 64;   // 16-byte loads per lane
        const int nm = wide ? TPB / 64 : 1;   // 64-block masks
        int k = 0;
        for (int w2 = 0; w2 < nm; ++w2)
        for (uint64_t dm = s_dmask[w2]; dm; ++k) {   // (wave-uniform)
            const uint32_t bit = (uint32_t)w2 * 64u + (uint32_t)(__ffsll((long long)dm) - 1);
            dm &= dm - 1;
            if ((k & (TPB / 64 - 1)) != wid) continue;
            const uint32_t blk = b0 + bit;
            const uint4* sl = reinterpret_cast<const uint4*>(tb.slots + ((uint64_t)blk << BLK_LOG2));
            uint4 e[NV];
#pragma unroll
            for (int q = 0; q < NV; ++q) e[q] = sl[lane + q * 64];
            uint64_t best = KEY_NONE, second = KEY_NONE;   // the block's two largest keys (top2_add)
            uint32_t live = 0;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                if (e[q].x && (int32_t)e[q].y > 0) {
                    top2_add(best, second, ((uint64_t)e[q].y << 32) | (uint32_t)(~e[q].x));
                    ++live;
                }
                if (e[q].z && (int32_t)e[q].w > 0) {
                    top2_add(best, second, ((uint64_t)e[q].w << 32) | (uint32_t)(~e[q].z));
                    ++live;
                }
            }
            wave_top2_u64(best, second, best, second);
            live = wave_sum_u32(live);
            if (lane == 0) {
                tb.bmax[blk] = best;
                tb.bmax2[blk] = second;
                tb.blive[blk] = live;
                tb.dirty[blk] = 0u;
                s_bm[bit] = best;
                s_bm2[bit] = second;
            }
        }
    }
    __syncthreads();
    if (part) {   // this workgroup's two largest keys, for sel_inline (part[2 wg], part[2 wg + 1])
        uint64_t best = 0ull, second = 0ull;
        if (threadIdx.x < 64) {
            best = s_bm[threadIdx.x];
            second = s_bm2[threadIdx.x];
            if (wide)   // one wave over the blocks past the first 64
                for (uint32_t i = threadIdx.x + 64u; i < per; i += 64u) top2_merge(best, second, s_bm[i], s_bm2[i]);
            wave_top2_u64(best, second, best, second);
            if (threadIdx.x == 0) {
                part[2 * blockIdx.x] = best;
                part[2 * blockIdx.x + 1] = second;
                if (finish == 2) KTR(5);
            }
        }
    }
}

// k_refresh in the form its grid needs: more than 64 table blocks per workgroup
// (the late grids of a large table) take the WIDE form
// (the grid is clamped to >= nblk / TPB: a workgroup re-maxes at most TPB blocks, one
// per thread, so a smaller grid would leave blocks' maxima stale)
#define GBPE_LAUNCH_REFRESH(S, grid, nblk, s, ...)                                                          \
    do {                                                                                                    \
        const uint32_t g_ = std::max<uint32_t>((uint32_t)(grid), (uint32_t)(((uint64_t)(nblk) + TPB - 1) / TPB)); \
        if ((uint64_t)g_ * 64u < (uint64_t)(nblk))                                                          \
            hipLaunchKernelGGL((k_refresh<S, true>), dim3(g_), dim3(TPB), 0, s, __VA_ARGS__);               \
        else                                                                                                \
            hipLaunchKernelGGL((k_refresh<S, false>), dim3(g_), dim3(TPB), 0, s, __VA_ARGS__);              \
    } while (0)

constexpr uint32_t GRP = 64;    // tiles per group sum (two-level tile prefix)
constexpr uint32_t GSTR = 64;   // group sums 256 B apart: each is its own atomic serialisation point

// argmax over block maxima + the reference's bpe_setup_merge (train.wgsl:340-364),
// by one workgroup of any size <= SEL_THREADS
__device__ void select_merge(DevState* st, Table tb, uint32_t* __restrict__ log, uint32_t* __restrict__ grpsum,
                             DevState* zst, uint32_t exact) {
    __shared__ uint64_t red[SEL_THREADS / 64];
    __shared__ uint32_t rlive[SEL_THREADS / 64];
    const uint32_t nt = blockDim.x;
    if (st->stop || st->sp_abort) return;
    {   // group sums of the coming stream pass (the zone's, when sector-sparse) start at zero
        const uint32_t ngrp = (uint32_t)gbpe_div_up(gbpe_div_up(zst ? zst->n : st->n, TILE), GRP);
        for (uint32_t g = threadIdx.x; g < ngrp; g += nt) grpsum[g * GSTR] = 0u;
    }
    uint64_t best = 0;
    uint32_t live = 0;
    for (uint32_t i = threadIdx.x; i < tb.nblk; i += nt) {
        uint64_t v = tb.bmax[i];
        best = v > best ? v : best;
        live += tb.blive[i];
    }
    best = wave_max_u64(best);
    live = wave_sum_u32(live);
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = best;
        rlive[threadIdx.x >> 6] = live;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (uint32_t w = 1; w < nt / 64; ++w) {
        best = red[w] > best ? red[w] : best;
        live += rlive[w];
    }
    st->live = live;
    if (live > st->max_live) st->max_live = live;
    st->ndirty = 0u;
    st->m = 0u;
    st->valid_total = 0u;
    const uint32_t mc = (uint32_t)(best >> 32);
    const uint32_t pid = ~(uint32_t)best;
    if (st->merges_done >= st->budget) {   // host asked for fewer merges this step
        return;
    }
    if (!zst && st->enter_lim && mc <= st->enter_lim && st->merges_done > 0u) {
        // counts fell far enough for the word-lexicon loop: end the step here so the
        // host enters it (C5's first count is 17 % of the stream, its second 0.6 %)
        return;
    }
    if (mc < 2u || st->next_id > 0xFFFFu) {   // train.wgsl:345-348
        st->stop = 1u;
        return;
    }
    if (zst && !exact) {
        // sector-sparse zone invariants: this merge's stale window
        // [new_n - m, new_n) of the previous stream lies in the zone's stale buffer
        // (n - 2mc >= Bp), and the zone stays >= 5 mc long so the next merge's window
        // does too (its count is <= mc + m <= 2 mc).  Otherwise the merge is not run
        // and the host returns to the dense loop.
        if ((uint64_t)(uint32_t)(st->n - st->Bp) < 2ull * mc) {
            // (cannot happen after the check below held)
            atomicOr(&st->err, ERR_SPARSE_WINDOW);
            st->stop = 1u;
            return;
        }
        if ((uint64_t)zst->n < 5ull * mc + 2u) {
            st->sp_abort = 1u;
            return;
        }
    }
    const uint32_t idx = table_find(tb, pid);
    if (idx == 0xFFFFFFFFu) {
        atomicOr(&st->err, ERR_PAIR_MISSING);
        st->stop = 1u;
        return;
    }
    tb.slots[idx].y = 0u;                  // every (a,b) occurrence is a merge site
    tb.dirty[idx >> BLK_LOG2] = 1u;
    const uint32_t d = st->merges_done;
    log[d * 4 + 0] = pid >> 16;
    log[d * 4 + 1] = pid & 0xFFFFu;
    log[d * 4 + 2] = st->next_id;
    log[d * 4 + 3] = mc;
    st->a = pid >> 16;
    st->b = pid & 0xFFFFu;
    st->nw = st->next_id;
    st->mc = mc;
    st->new_n = st->n - mc;
    if (zst) {   // the zone's view of the merge: k_delta / k_compact run on it unchanged
        zst->a = st->a;
        zst->b = st->b;
        zst->nw = st->nw;
        zst->mc = mc;
        zst->new_n = exact ? zst->n : zst->n - mc;   // zone keep limit: global new_n - B
        zst->m = 0u;
        zst->valid_total = 0u;
        zst->merges_done = d + 1u;
        st->body_rm = 0u;
        st->cand = 0u;
        st->hitsec = 0u;
    }
    st->next_id += 1u;
    st->epoch += 1u;
    st->merges_done = d + 1u;
}

__global__ __launch_bounds__(SEL_THREADS) void k_select(DevState* st, Table tb, uint32_t* __restrict__ log,
                                                        uint32_t* __restrict__ grpsum, DevState* zst, uint32_t exact) {
    select_merge(st, tb, log, grpsum, zst, exact);
}

// the next merge's count (the table maximum): the sparse entry decision before any merge ran
__global__ __launch_bounds__(1024) void k_topcount(Table tb, uint32_t* __restrict__ out) {
    __shared__ uint64_t red[16];
    uint64_t best = 0;
    for (uint32_t i = threadIdx.x; i < tb.nblk; i += 1024) {
        const uint64_t v = tb.bmax[i];
        best = v > best ? v : best;
    }
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) best = red[w] > best ? red[w] : best;
        *out = (uint32_t)(best >> 32);
    }
}

// live pairs (count > 0) from the per-block live counts k_refresh keeps, once per
// sparse step (the dense loop's k_select counts them every merge)
__global__ __launch_bounds__(1024) void k_live(DevState* st, Table tb) {
    __shared__ uint32_t red[16];
    uint32_t live = 0;
    for (uint32_t i = threadIdx.x; i < tb.nblk; i += 1024) live += tb.blive[i];
    live = wave_sum_u32(live);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) live += red[w];
        st->live = live;
        if (live > st->max_live) st->max_live = live;
    }
}

// Step boundaries without copy engines: the host's four 4-byte resets and its
// three read-backs (state, zone state, merge log) were each a blit on the
// stream (~5 us apiece with their gaps, ~40 us per step); one thread sets the
// counters, and one workgroup writes the read-backs straight into the pinned
// host buffers (vector stores to host memory, a system-scope fence at the end).
__global__ void k_step_in(DevState* st, DevState* zst, uint32_t k) {
    st->merges_done = 0u;
    st->budget = k;
    if (zst) {
        zst->merges_done = 0u;
        st->sel_round = 0u;
    }
}

__global__ __launch_bounds__(1024) void k_step_out(DevState* st, DevState* zst, Table tb, int live_too,
                                                   const uint32_t* __restrict__ log, uint32_t nlog,
                                                   const uint32_t* __restrict__ clog, uint32_t nclog,
                                                   DevState* h_st, DevState* h_zst, uint32_t* h_log, uint32_t* h_clog) {
    constexpr int NW = sizeof(DevState) / 4;
    static_assert(NW <= 1024, "DevState fits one pass");
    __shared__ uint32_t red[16];
    __shared__ union {
        DevState d;
        uint32_t w[NW];
    } g;
    const uint32_t t = threadIdx.x;
    uint32_t live = 0;
    if (live_too) {   // k_live: live pairs from the per-block live counts (16-byte loads, 4 in flight)
        const uint32_t nq = tb.nblk / 4u;
        const uint4* bq = reinterpret_cast<const uint4*>(tb.blive);
        if (4u * nq + t < tb.nblk) live += tb.blive[4u * nq + t];
        for (uint32_t i = t; i < nq; i += 4096) {
            uint4 q[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = i + k * 1024u < nq ? bq[i + k * 1024u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int k = 0; k < 4; ++k) live += q[k].x + q[k].y + q[k].z + q[k].w;
        }
        live = wave_sum_u32(live);
        if ((t & 63) == 0) red[t >> 6] = live;
    }
    if (t < (uint32_t)NW) g.w[t] = reinterpret_cast<const uint32_t*>(st)[t];
    __syncthreads();
    if (live_too && t == 0) {
        for (int w = 1; w < 16; ++w) live += red[w];
        g.d.live = live;
        if (live > g.d.max_live) g.d.max_live = live;
        st->live = g.d.live;
        st->max_live = g.d.max_live;
    }
    __syncthreads();
    if (t < (uint32_t)NW) reinterpret_cast<uint32_t*>(h_st)[t] = g.w[t];
    if (zst && t < (uint32_t)NW) reinterpret_cast<uint32_t*>(h_zst)[t] = reinterpret_cast<const uint32_t*>(zst)[t];
    for (uint32_t i = t; i < nlog; i += 1024) h_log[i] = log[i];
    for (uint32_t i = t; i < nclog; i += 1024) h_clog[i] = clog[i];
    __threadfence_system();
}

// A merge is "active" for the stream kernels iff k_select logged it this round.
__device__ __forceinline__ bool merge_active(const DevState* st, uint32_t round) {
    return !st->stop && st->merges_done == round + 1u;
}

template <typename S>
__device__ __forceinline__ void load_own(const S* cur, uint64_t i0, uint32_t* __restrict__ x) {
    constexpr int V = EPT * sizeof(S) / 16;
    uint4 v[V];
    const uint4* src = reinterpret_cast<const uint4*>(cur + i0);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = src[k];
    const S* e = reinterpret_cast<const S*>(v);
#pragma unroll
    for (int k = 0; k < EPT; ++k) x[k] = e[k];
}

constexpr int LTAB_T = 1024;          // per-workgroup LDS delta table of k_body / the zone pass
constexpr int LTAB_Z = 4096;          // k_delta on a sparse zone: its stale tail holds many distinct pairs


__device__ __forceinline__ uint32_t lane_mask32(uint64_t i0, uint64_t lim) {
    // bits k with i0 + k < lim, k < 32
    return i0 >= lim ? 0u : (i0 + 32 <= lim ? 0xFFFFFFFFu : ((1u << (uint32_t)(lim - i0)) - 1u));
}

// ── two-stage delta reduction of the multi-tile zone passes ─────────────────
// Early merges (zones of 10^6-10^8 symbols) produce their count deltas in
// thousands of workgroups, each holding thousands of distinct pairs in its LDS
// table; flushing every table into the global table was most of an early
// merge's time (a diagnostic build without the stale-tail flush: 250 -> 33 us per
// merge at merges 10-18, 1 GiB): the same hot pairs, one contended global atomic
// per pair per workgroup.  Instead each workgroup DUMPS its table, partitioned
// by pair hash into ZDR_P buckets (plain stores, no atomics), and k_zdr — one
// workgroup per bucket — aggregates its bucket of every dump in LDS and adds each
// distinct pair to the global table once.
constexpr uint32_t ZDR_P = 256;          // hash buckets = k_zdr workgroups
constexpr int ZDR_N_TILE = LTAB_Z;       // dump capacity of a zone tile workgroup (its LDS table)
constexpr int ZDR_N_CHURN = 8192;        // ... of a k_churn workgroup
constexpr int ZDR_R = 4096;              // k_zdr's LDS table
__device__ __forceinline__ uint32_t zdr_part(uint32_t pid) { return gbpe_fmix32(pid ^ 0x85EBCA6Bu) >> 24; }

struct ZdrView {                 // where stage-1 workgroup w writes (host-sized); out == null: flush instead
    uint2* out = nullptr;        // entries: w < ntile ? w * ZDR_N_TILE : ntile * ZDR_N_TILE + (w - ntile) * ZDR_N_CHURN
    uint32_t* offs = nullptr;    // (ZDR_P + 1) bucket offsets per workgroup
    uint32_t* flag = nullptr;    // = tag when workgroup w dumped this merge
    uint32_t ntile = 0;          // tile workgroups before the churn workgroups
    uint32_t tag = 0;            // unique per merge
};
__device__ __forceinline__ uint64_t zdr_base(const ZdrView& z, uint32_t w) {
    return w < z.ntile ? (uint64_t)w * ZDR_N_TILE
                       : (uint64_t)z.ntile * ZDR_N_TILE + (uint64_t)(w - z.ntile) * ZDR_N_CHURN;
}

// stage 1: workgroup w's LDS table (its live entries) to its dump, bucket by bucket
template <int N>
__device__ void lds_dump(LdsTab<N>& t, const ZdrView& z, uint32_t w) {
    __shared__ uint32_t s_cnt[ZDR_P];
    __shared__ uint32_t s_tot;
    const uint32_t nt = blockDim.x, tid = threadIdx.x;
    __syncthreads();   // every lds_add of the table is done
    for (uint32_t p = tid; p < ZDR_P; p += nt) s_cnt[p] = 0u;
    __syncthreads();
    for (uint32_t i = tid; i < (uint32_t)N; i += nt) {
        const uint32_t k = t.key[i];
        if (k && t.val[i]) atomicAdd(&s_cnt[zdr_part(k)], 1u);
    }
    __syncthreads();
    if (tid < 64) {   // exclusive scan of the bucket counts by one wave (4 per lane)
        uint32_t c[ZDR_P / 64], sum = 0;
#pragma unroll
        for (int q = 0; q < (int)(ZDR_P / 64); ++q) {
            c[q] = s_cnt[tid * (ZDR_P / 64) + q];
            sum += c[q];
        }
        const uint32_t incl = wave_scan_incl_u32(sum);
        uint32_t run = incl - sum;
        uint32_t* offs = z.offs + (uint64_t)w * (ZDR_P + 1);
#pragma unroll
        for (int q = 0; q < (int)(ZDR_P / 64); ++q) {
            const uint32_t p = tid * (ZDR_P / 64) + q;
            s_cnt[p] = run;
            offs[p] = run;
            run += c[q];
        }
        if (tid == 63) {
            offs[ZDR_P] = run;
            s_tot = run;
        }
    }
    __syncthreads();
    if (s_tot == 0u) return;   // (block-uniform) nothing to dump: the flag stays stale
    uint2* out = z.out + zdr_base(z, w);
    for (uint32_t i = tid; i < (uint32_t)N; i += nt) {
        const uint32_t k = t.key[i], v = t.val[i];
        if (k && v) out[atomicAdd(&s_cnt[zdr_part(k)], 1u)] = make_uint2(k, v);
    }
    if (tid == 0) z.flag[w] = z.tag;   // (read by k_zdr, a later launch)
}

// Pass 1 (one tile of TILE symbols per workgroup): merge-site mask, survivor
// count per tile, count deltas.
//   hit(i)  = (i >= 1) && !ws(i) && tok(i-1) == a && tok(i) == b     (B-side, train.wgsl:491-497)
//   rw(i)   = hit(i+1)                                               (A-side, train.wgsl:482-485)
//   survivor(i) = !hit(i)
// Old pair at i is destroyed iff hit(i-1)|hit(i)|hit(i+1) or i >= limit (stale tail);
// new pair at a survivor i < limit: hit(i-1) → (nw, tok'(i)); else hit(i+1) → (tok(i-1), nw).
// The tile (32 symbols per lane + the 2 before + 1 after) is loaded before the
// loop state is read, so the state's scalar load overlaps the HBM latency.  Lanes
// with no site within reach and no tail element do no delta work; a tile with no
// such lane passes a single barrier.
// STAGE (the sector-sparse zone: few tiles, latency-bound): the work loop reads
// the lane's symbols from an LDS copy instead of re-reading L2 per position.
template <typename S, bool EXACT, bool STAGE = false>
__global__ __launch_bounds__(TPB) void k_delta(DevState* st, uint32_t round, const S* cur, Table tb,
                                               uint32_t* __restrict__ hitmask, uint32_t* __restrict__ tile_cnt,
                                               uint32_t* __restrict__ grpsum, uint32_t eager_tiles,
                                               uint32_t ngroups = 0xFFFFFFFFu, ZdrView zv = ZdrView()) {
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    __shared__ LdsTab<STAGE ? LTAB_Z : LTAB_T> lt;
    __shared__ uint32_t stg[STAGE ? EPT * TPB : 1];
    __shared__ uint32_t red[TPB / 64], s_workw[TPB / 64];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t tl = blockIdx.x;
    if (tl >= ngroups) {   // a stale-tail slice block (as in k_delta_mt); tiles skip their tail loop
        const uint4 s0 = reinterpret_cast<const uint4*>(st)[0];
        const uint4 s1 = reinterpret_cast<const uint4*>(st)[1];
        const uint2 s2 = reinterpret_cast<const uint2*>(st)[4];
        const uint32_t n = s0.x, lim = s1.w, pid_ab = (s0.w << 16) | s1.x;
        if (EXACT || s0.y || s2.y != round + 1u || n <= lim) return;
        const uint32_t nt2 = gridDim.x - ngroups, q = tl - ngroups;
        const uint32_t len = n - lim, per = (len + nt2 - 1) / nt2;
        const uint64_t a0 = (uint64_t)lim + (uint64_t)q * per;
        const uint64_t a1 = a0 + per < (uint64_t)n ? a0 + per : (uint64_t)n;
        if (a0 >= a1) return;
        lds_clear(lt);
        __syncthreads();
        for (uint64_t i = a0 + t; i < a1; i += TPB) {
            if (i == 0) continue;
            const uint32_t xi = cur[i];
            if (xi & WS) continue;
            const uint32_t tp = cur[i - 1] & TM, ti = xi & TM;
            if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
        }
        lds_flush(lt, tb, st);
        return;
    }
    // tiles past the host's view of the stream (a shard that may have grown by an
    // appended window) check the length before loading anything
    if (tl >= eager_tiles && (uint64_t)tl * TILE >= st->n) return;
    const uint64_t base = (uint64_t)tl * TILE;
    const uint64_t i0 = base + (uint64_t)t * EPT;
    // loads first, unconditionally (buffers are padded: every launched tile is in
    // bounds); the compiler barrier keeps them ahead of the state's scalar loads
    // so both round trips overlap
    uint32_t x[EPT];
    uint32_t lh = 0, rh = 0;
    {
        const uint64_t hi = i0 >= 2 ? i0 - 2 : 0;
        if (sizeof(S) == 2) {
            lh = *reinterpret_cast<const uint32_t*>(cur + hi);
        } else {
            const uint2 v2 = *reinterpret_cast<const uint2*>(cur + hi);
            lh = v2.x;
            rh = v2.y;
        }
    }
    const uint32_t nxr = (uint32_t)cur[i0 + EPT];
    load_own(cur, i0, x);
    // the loop state, one snapshot: fields n .. merges_done (DevState offsets 0..39)
    const uint4 s0 = reinterpret_cast<const uint4*>(st)[0];   // n, stop, next_id, a
    const uint4 s1 = reinterpret_cast<const uint4*>(st)[1];   // b, nw, mc, new_n
    const uint2 s2 = reinterpret_cast<const uint2*>(st)[4];   // m, merges_done
    asm volatile("" ::: "memory");
    const uint32_t n = s0.x, a = s0.w, b = s1.x, nw = s1.y, new_n = s1.w;
    const uint32_t ntiles = (uint32_t)gbpe_div_up(n, TILE);
    if (s0.y || s2.y != round + 1u || tl >= ntiles) return;   // merge_active()
    const uint32_t pid_ab = (a << 16) | b;
    const uint32_t lim = EXACT ? 0xFFFFFFFFu : new_n;
    uint32_t xm2 = sizeof(S) == 2 ? (lh & 0xFFFFu) : lh;   // symbol at i0 - 2
    uint32_t xm1 = sizeof(S) == 2 ? (lh >> 16) : rh;       // symbol at i0 - 1
    if (i0 < 2) xm2 = xm1 = 0;                              // tokens are never 0 = a, b
    // branch-free site detection: eb bit j = (x_j == b) (a B-side symbol carries no
    // word-start bit), ea bit j = (tok(x_j) == a)
    uint32_t eb = 0, ea = 0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        eb |= (x[k] == b ? 1u : 0u) << k;
        ea |= ((x[k] & TM) == a ? 1u : 0u) << k;
    }
    const uint32_t inb = lane_mask32(i0, n);
    const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a ? 1u : 0u)) & inb;   // hit(i0 + j)
    const uint32_t h_m1 = (xm1 == b && (xm2 & TM) == a && i0 - 1 < n) ? 1u : 0u;  // hit(i0 - 1)
    const uint32_t h_32 = (nxr == b && (ea >> (EPT - 1)) && i0 + EPT < n) ? 1u : 0u;  // hit(i0 + EPT)
    const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_32 << (EPT + 1));
    uint32_t cnt = __popc(inb & ~hitm);
    uint32_t tail = 0;
    const bool work = hbits != 0 || (i0 + EPT > lim && i0 < n);
    cnt = wave_sum_u32(cnt);
    const bool wave_work = __any(work);
    if (lane == 0) {
        red[wid] = cnt;
        s_workw[wid] = wave_work;
    }
    __syncthreads();
    if (s_workw[0] | s_workw[1] | s_workw[2] | s_workw[3]) {   // block-uniform: only tiles with a site or a tail element touch the table
        lds_clear(lt);
        __syncthreads();
        if (STAGE && work) {
#pragma unroll
            for (int k = 0; k < EPT; ++k) stg[k * TPB + t] = x[k];
        }
        if (work) {
            // only the positions where a pair can change: within one of a site, or in
            // the stale tail; symbols re-read from the (L1/L2-hot) tile by index so the
            // register window is never dynamically indexed
            const uint32_t below = lane_mask32(i0, lim);
            tail = __popc(inb & ~hitm & ~below);
            // positions next to a site below the keep limit; the stale tail (old pairs
            // destroyed, nothing new) is spread over the whole workgroup below
            uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
            while (rel) {
                const int k = __ffs(rel) - 1;
                rel &= rel - 1;
                const uint64_t i = i0 + k;
                if (i == 0) continue;
                uint32_t xi, xp;
                if (STAGE) {   // the lane's own symbols, staged in LDS below
                    xi = stg[k * TPB + t];
                    xp = k ? stg[(k - 1) * TPB + t] : xm1;
                } else {   // L1/L2-hot re-read (keeps the streaming kernel's LDS small)
                    xi = cur[i];
                    xp = cur[i - 1];
                }
                if (xi & WS) continue;   // no pair ends at i (old or new)
                const bool hm = (hbits >> k) & 1u, h0 = (hbits >> (k + 1)) & 1u, hp = (hbits >> (k + 2)) & 1u;
                const uint32_t tp = xp & TM, ti = xi & TM;
                if (tp && ti) {
                    const uint32_t pid = (tp << 16) | ti;
                    if (pid != pid_ab) lds_add(lt, tb, st, pid, 0xFFFFFFFFu);   // old pair destroyed
                }
                if (!h0 && i < lim) {
                    if (hm) {
                        const uint32_t t2 = hp ? nw : ti;
                        if (t2) lds_add(lt, tb, st, (nw << 16) | t2, 1u);
                    } else if (hp && tp) {
                        lds_add(lt, tb, st, (tp << 16) | nw, 1u);
                    }
                }
            }
        }
        if (!EXACT && ngroups == 0xFFFFFFFFu && (uint64_t)base + TILE > lim && base < n) {
            const uint64_t hi = (uint64_t)n < base + TILE ? (uint64_t)n : base + TILE;
            for (uint64_t i = (lim > base ? (uint64_t)lim : base) + t; i < hi; i += TPB) {
                if (i == 0) continue;
                const uint32_t xi = cur[i];
                if (xi & WS) continue;
                const uint32_t tp = cur[i - 1] & TM, ti = xi & TM;
                if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
            }
        }
        if (zv.out) lds_dump(lt, zv, tl);   // multi-tile zone pass: k_zdr adds the deltas
        else lds_flush(lt, tb, st);
        tail = wave_sum_u32(tail);
        if (lane == 0 && tail) atomicAdd(&st->m, tail);
    }
    // stores last: nothing waits on them
    if (i0 < n) hitmask[(uint64_t)tl * TPB + t] = hitm;
    if (t == 0) {
        const uint32_t tot = red[0] + red[1] + red[2] + red[3];
        tile_cnt[tl] = tot;
        atomicAdd(&grpsum[(tl / GRP) * GSTR], tot);
    }
}

// k_delta over TPW consecutive tiles per workgroup, one LDS delta table for all
// of them, flushed once: the dense loop's early merges (10^5-10^6 sites) add to
// the same hot pairs from every tile, and same-address device atomics serialise
// at the memory side, so TPW x fewer flushes is TPW x fewer of them.  Same
// per-tile outputs and delta rule as k_delta.
template <typename S, bool EXACT, int DELTA_TPW>
__global__ __launch_bounds__(TPB) void k_delta_mt(DevState* st, uint32_t round, const S* cur, Table tb,
                                                  uint32_t* __restrict__ hitmask, uint32_t* __restrict__ tile_cnt,
                                                  uint32_t* __restrict__ grpsum, uint32_t eager_tiles, uint32_t ngroups,
                                                  uint32_t first_block = 0, ZdrView zv = ZdrView()) {
    if (blockIdx.x < first_block) return;   // (split launches: tiles and tail apart)
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    __shared__ LdsTab<LTAB_Z> lt;
    __shared__ uint32_t red[TPB / 64];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint4 s0 = reinterpret_cast<const uint4*>(st)[0];   // n, stop, next_id, a
    const uint4 s1 = reinterpret_cast<const uint4*>(st)[1];   // b, nw, mc, new_n
    const uint2 s2 = reinterpret_cast<const uint2*>(st)[4];   // m, merges_done
    const uint32_t n = s0.x, a = s0.w, b = s1.x, nw = s1.y, new_n = s1.w;
    const uint32_t ntiles = (uint32_t)gbpe_div_up(n, TILE);
    if (s0.y || s2.y != round + 1u) return;   // merge_active()
    const uint32_t pid_ab = (a << 16) | b;
    const uint32_t lim = EXACT ? 0xFFFFFFFFu : new_n;
    lds_clear(lt);
    __syncthreads();
    if (blockIdx.x >= ngroups) {
        // stale tail [new_n, n): every old pair there is destroyed.  Blocks past
        // the tile groups take one contiguous slice each (up to ~2K symbols, so
        // their LDS table holds every distinct pair), instead of the few tile
        // workgroups the tail falls in walking all of it with an overflowing table.
        if (EXACT || n <= lim) return;
        const uint32_t nt2 = gridDim.x - ngroups, q = blockIdx.x - ngroups;
        const uint32_t len = n - lim, per = (len + nt2 - 1) / nt2;
        const uint64_t a0 = (uint64_t)lim + (uint64_t)q * per;
        const uint64_t a1 = a0 + per < (uint64_t)n ? a0 + per : (uint64_t)n;
        if (a0 >= a1) return;   // block-uniform
        for (uint64_t i = a0 + t; i < a1; i += TPB) {
            if (i == 0) continue;
            const uint32_t xi = cur[i];
            if (xi & WS) continue;
            const uint32_t tp = cur[i - 1] & TM, ti = xi & TM;
            if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
        }
        lds_flush(lt, tb, st);
        return;
    }
    uint32_t tail = 0;
    for (int q = 0; q < DELTA_TPW; ++q) {
        const uint32_t tl = blockIdx.x * DELTA_TPW + q;
        if (tl >= ntiles || (tl >= eager_tiles && (uint64_t)tl * TILE >= n)) break;   // block-uniform
        const uint64_t base = (uint64_t)tl * TILE;
        const uint64_t i0 = base + (uint64_t)t * EPT;
        uint32_t x[EPT];
        uint32_t lh = 0, rh = 0;
        {
            const uint64_t hi = i0 >= 2 ? i0 - 2 : 0;
            if (sizeof(S) == 2) {
                lh = *reinterpret_cast<const uint32_t*>(cur + hi);
            } else {
                const uint2 v2 = *reinterpret_cast<const uint2*>(cur + hi);
                lh = v2.x;
                rh = v2.y;
            }
        }
        const uint32_t nxr = (uint32_t)cur[i0 + EPT];
        load_own(cur, i0, x);
        uint32_t xm2 = sizeof(S) == 2 ? (lh & 0xFFFFu) : lh;
        uint32_t xm1 = sizeof(S) == 2 ? (lh >> 16) : rh;
        if (i0 < 2) xm2 = xm1 = 0;
        uint32_t eb = 0, ea = 0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            eb |= (x[k] == b ? 1u : 0u) << k;
            ea |= ((x[k] & TM) == a ? 1u : 0u) << k;
        }
        const uint32_t inb = lane_mask32(i0, n);
        const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a ? 1u : 0u)) & inb;
        const uint32_t h_m1 = (xm1 == b && (xm2 & TM) == a && i0 - 1 < n) ? 1u : 0u;
        const uint32_t h_32 = (nxr == b && (ea >> (EPT - 1)) && i0 + EPT < n) ? 1u : 0u;
        const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_32 << (EPT + 1));
        uint32_t cnt = __popc(inb & ~hitm);
        cnt = wave_sum_u32(cnt);
        if (hbits != 0 || (i0 + EPT > lim && i0 < n)) {
            const uint32_t below = lane_mask32(i0, lim);
            tail += __popc(inb & ~hitm & ~below);
            uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
            while (rel) {
                const int k = __ffs(rel) - 1;
                rel &= rel - 1;
                const uint64_t i = i0 + k;
                if (i == 0) continue;
                const uint32_t xi = cur[i], xp = cur[i - 1];
                if (xi & WS) continue;
                const bool hm = (hbits >> k) & 1u, h0 = (hbits >> (k + 1)) & 1u, hp = (hbits >> (k + 2)) & 1u;
                const uint32_t tp = xp & TM, ti = xi & TM;
                if (tp && ti) {
                    const uint32_t pid = (tp << 16) | ti;
                    if (pid != pid_ab) lds_add(lt, tb, st, pid, 0xFFFFFFFFu);
                }
                if (!h0 && i < lim) {
                    if (hm) {
                        const uint32_t t2 = hp ? nw : ti;
                        if (t2) lds_add(lt, tb, st, (nw << 16) | t2, 1u);
                    } else if (hp && tp) {
                        lds_add(lt, tb, st, (tp << 16) | nw, 1u);
                    }
                }
            }
        }
        // (the stale tail's destroyed pairs: the tail blocks above)
        if (i0 < n) hitmask[(uint64_t)tl * TPB + t] = hitm;
        if (lane == 0) red[wid] = cnt;
        __syncthreads();
        if (t == 0) {
            const uint32_t tot = red[0] + red[1] + red[2] + red[3];
            tile_cnt[tl] = tot;
            atomicAdd(&grpsum[(tl / GRP) * GSTR], tot);
        }
        __syncthreads();   // red[] is rewritten by the next tile
    }
    if (zv.out) lds_dump(lt, zv, blockIdx.x);   // multi-tile zone pass: k_zdr adds the deltas
    else lds_flush(lt, tb, st);
    tail = wave_sum_u32(tail);
    if (lane == 0 && tail) atomicAdd(&st->m, tail);
}

// Pass 2.  Blocks [0, ntiles): in-place A-side rewrite (train.wgsl:486-487) +
// scatter of the survivors with old index < new_n (the reference bound,
// train.wgsl:727; all of them with EXACT) at tile prefix = group sums + the
// tile counts of this group before the tile.  Blocks >= ntiles (reference
// compaction only): the stale tail window [new_n - m, new_n) of the new
// stream — add its pairs to the count table.
constexpr int CTPB = 512;             // k_compact threads per tile
constexpr int CEPT = TILE / CTPB;     // 16 symbols per k_compact thread

template <typename S, int E>
__device__ __forceinline__ void load_own_n(const S* __restrict__ cur, uint64_t i0, uint32_t* __restrict__ x) {
    constexpr int V = E * sizeof(S) / 16;
    uint4 v[V];
    const uint4* src = reinterpret_cast<const uint4*>(cur + i0);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = src[k];
    const S* e = reinterpret_cast<const S*>(v);
#pragma unroll
    for (int k = 0; k < E; ++k) x[k] = e[k];
}

// ZONE (sector-sparse loop): st is the zone's view; the stale window is not in
// place in `oth` (the zone's coordinates shift with the body) but copied to `win`
// by k_body before this pass: window symbol j = win[mc - m + j], stored at zone
// position (zone survivors - m) + j.  gst is the global state (count check).
template <typename S, bool EXACT, bool ZONE = false>
__global__ __launch_bounds__(CTPB) void k_compact(DevState* st, uint32_t round, S* __restrict__ cur, S* __restrict__ oth,
                                                 const uint32_t* __restrict__ hitmask,
                                                 const uint32_t* __restrict__ tile_cnt,
                                                 const uint32_t* __restrict__ grpsum, Table tb,
                                                 const S* __restrict__ win = nullptr, const DevState* gst = nullptr,
                                                 uint32_t split = 0) {
    // split launches: 1 = tile blocks only, 2 = every block a window block
    // one LDS arena: the compaction stage of tile blocks or the delta table of tail blocks
    constexpr int STAGE = (TILE + 16) * sizeof(S);
    constexpr int ARENA = (sizeof(LdsTab<LTAB>) > STAGE ? sizeof(LdsTab<LTAB>) : STAGE) / 16;
    __shared__ uint4 arena[ARENA];
    __shared__ uint32_t wsum[CTPB / 64], psum[CTPB / 64];
    S* stage = reinterpret_cast<S*>(arena);
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t tl = blockIdx.x;
    const uint64_t base = (uint64_t)tl * TILE;
    if (!merge_active(st, round)) return;
    const uint32_t n = st->n, new_n = st->new_n, nw = st->nw;
    const uint32_t limit = EXACT ? n : new_n;
    const uint32_t ntiles = (uint32_t)gbpe_div_up(n, TILE);
    if (split == 1 && tl >= ntiles) return;
    if (tl >= ntiles || split == 2) {
        if (EXACT) return;
        // ── stale tail window ──
        const uint32_t m = st->m;
        if (m == 0) return;
        LdsTab<LTAB>& lt = *reinterpret_cast<LdsTab<LTAB>*>(arena);
        __shared__ uint32_t left_val;
        lds_clear(lt);
        uint32_t lo = new_n - m;
        const uint32_t tb0 = split == 2 ? tl : tl - ntiles, ntb = split == 2 ? gridDim.x : gridDim.x - ntiles;
        uint32_t woff = 0;
        if (ZONE) {   // window start = zone survivors - m (the group sums hold the survivors)
            __shared__ uint32_t s_surv[CTPB / 64];
            const uint32_t ngrp = (uint32_t)gbpe_div_up(ntiles, GRP);
            uint32_t sv = 0;
            for (uint32_t g = t; g < ngrp; g += CTPB) sv += grpsum[g * GSTR];
            sv = wave_sum_u32(sv);
            if (lane == 0) s_surv[wid] = sv;
            __syncthreads();
            sv = 0;
            for (int w2 = 0; w2 < CTPB / 64; ++w2) sv += s_surv[w2];
            lo = sv - m;
            woff = st->mc - m;
        }
        const uint32_t hi = lo + m;
        if (tb0 == 0 && wid == 0 && lo >= 1) {
            // the survivor just before the window: last j < new_n with hit(j) == 0; its
            // value is the A-side-rewritten symbol (the rewrite is idempotent, so racing
            // with a tile block's in-place write is harmless)
            int64_t wi = (int64_t)(new_n - 1) / 32;
            uint32_t found = 0xFFFFFFFFu;
            while (wi >= 0 && found == 0xFFFFFFFFu) {
                const int64_t mywi = wi - lane;
                uint32_t inv = 0;
                if (mywi >= 0) {
                    const uint64_t wbase = (uint64_t)mywi * 32;
                    inv = ~hitmask[mywi] & lane_mask32(wbase, new_n);   // survivors below new_n
                }
                const unsigned long long has = __ballot(inv != 0u);
                if (has) {
                    const int l = __ffsll((long long)has) - 1;   // lowest lane = largest word index
                    const uint32_t inv_l = (uint32_t)__builtin_amdgcn_readlane(inv, l);
                    found = (uint32_t)((wi - l) * 32 + (31 - __clz(inv_l)));
                }
                wi -= 64;
            }
            if (lane == 0) {
                uint32_t v = 0;
                if (found != 0xFFFFFFFFu) {
                    v = cur[found];
                    const uint32_t f1 = found + 1;
                    const bool rw = (f1 < n) && ((hitmask[f1 / 32] >> (f1 % 32)) & 1u);
                    if (rw) v = nw | (v & WS);
                }
                left_val = v;
            }
        }
        __syncthreads();
        for (uint32_t d = lo + tb0 * CTPB + t; d < hi; d += ntb * CTPB) {
            if (d == 0) continue;
            uint32_t x0, x1;
            if (ZONE) {
                x1 = win[woff + (d - lo)];
                x0 = (d == lo) ? left_val : (uint32_t)win[woff + (d - lo) - 1];
                oth[d] = (S)x1;
            } else {
                x0 = (d == lo) ? left_val : (uint32_t)oth[d - 1];
                x1 = oth[d];
            }
            const uint32_t t0 = x0 & TM, t1 = x1 & TM;
            if (!(x1 & WS) && t0 && t1) lds_add(lt, tb, st, (t0 << 16) | t1, 1u);
        }
        lds_flush(lt, tb, st);
        return;
    }
    // 512 threads x 16 symbols cover the 8192-symbol tile; every independent load
    // first: prefix terms, mask word, the tile
    const uint64_t j0 = base + (uint64_t)t * CEPT;
    const uint32_t G = tl / GRP;
    uint32_t part = 0;
    {
        const uint32_t j = G * GRP + t;
        const uint32_t v0 = (t < (int)GRP && j < tl) ? tile_cnt[j] : 0u;
        const uint32_t g0 = ((uint32_t)t < G) ? grpsum[t * GSTR] : 0u;
        const uint32_t g1 = ((uint32_t)t + CTPB < G) ? grpsum[(t + CTPB) * GSTR] : 0u;
        part = v0 + g0 + g1;
    }
    const uint32_t hw = hitmask[(uint64_t)tl * TPB + (t >> 1)];
    const uint32_t hn = (t & 1) ? hitmask[(uint64_t)tl * TPB + (t >> 1) + 1] : 0u;   // may be the next tile's first word
    uint32_t x[CEPT];
    load_own_n<S, CEPT>(cur, j0, x);
    for (uint32_t g = t + 2 * CTPB; g < G; g += CTPB) part += grpsum[g * GSTR];   // only past 2*CTPB groups
    const uint32_t hm = (t & 1) ? (hw >> 16) : (hw & 0xFFFFu);
    const uint32_t nb = (t & 1) ? (hn & 1u) : ((hw >> 16) & 1u);
    const uint32_t inb = lane_mask32(j0, n) & 0xFFFFu;
    const uint32_t nextbit = (j0 + CEPT < n) ? nb : 0u;
    const uint32_t rwm = ((hm >> 1) | (nextbit << (CEPT - 1))) & inb;
    const uint32_t valid = inb & ~hm;
    const uint32_t keep = EXACT ? valid : (valid & lane_mask32(j0, limit));
    if (rwm) {   // in-place A-side rewrite (train.wgsl:486-487): the reference's ping buffer
#pragma unroll
        for (int k = 0; k < CEPT; ++k) {
            if ((rwm >> k) & 1u) {
                x[k] = nw | (x[k] & WS);
                cur[j0 + k] = (S)x[k];
            }
        }
    }
    const uint32_t cnt = __popc(keep);
    // block exclusive scan of cnt + block sum of part
    const uint32_t incl = wave_scan_incl_u32(cnt);
    part = wave_sum_u32(part);
    if (lane == 63) wsum[wid] = incl;
    if (lane == 0) psum[wid] = part;
    __syncthreads();
    uint32_t pre = incl - cnt, total = 0, prefix = 0;
#pragma unroll
    for (int w2 = 0; w2 < CTPB / 64; ++w2) {
        pre += w2 < wid ? wsum[w2] : 0u;
        total += wsum[w2];
        prefix += psum[w2];
    }
    if (tl == ntiles - 1 && t == 0 &&
        prefix + tile_cnt[tl] != (ZONE ? gst->new_n - (gst->B - gst->body_rm) : new_n))
        atomicOr(ZONE ? (uint32_t*)&gst->err : &st->err, ERR_COUNT_MISMATCH);
    // stage at the destination's alignment phase so both sides move whole 16-byte words
    constexpr uint32_t VE = 16 / sizeof(S);           // symbols per 16-byte word
    const uint32_t ph = prefix & (VE - 1);
    pre += ph;
#pragma unroll
    for (int k = 0; k < CEPT; ++k)
        if ((keep >> k) & 1u) stage[pre++] = (S)x[k];
    __syncthreads();
    S* dst = oth + (prefix - ph);                      // 16-byte aligned
    const uint32_t end = ph + total;
    const uint32_t nvec = end / VE;
    uint4* dv = reinterpret_cast<uint4*>(dst);
    const uint4* sv = reinterpret_cast<const uint4*>(stage);
    for (uint32_t v = t; v < nvec; v += CTPB) {
        if (v == 0 && ph) {
            for (uint32_t j = ph; j < VE && j < end; ++j) dst[j] = stage[j];   // partial head word
        } else {
            dv[v] = sv[v];
        }
    }
    if (t == 0 && nvec * VE < end) {
        for (uint32_t j = (nvec * VE > ph ? nvec * VE : ph); j < end; ++j) dst[j] = stage[j];   // partial tail word
    }
}

// stage 2: bucket p of every dump of this merge, aggregated, into the global table
__global__ __launch_bounds__(TPB) void k_zdr(ZdrView z, uint32_t nd, Table tb, DevState* st, uint32_t round) {
    __shared__ LdsTab<ZDR_R> lt;
    if (!merge_active(st, round)) return;
    lds_clear(lt);
    __syncthreads();
    const uint32_t p = blockIdx.x;
    for (uint32_t w = threadIdx.x; w < nd; w += TPB) {
        if (z.flag[w] != z.tag) continue;
        const uint32_t* offs = z.offs + (uint64_t)w * (ZDR_P + 1);
        const uint32_t b = offs[p], e = offs[p + 1];
        const uint2* in = z.out + zdr_base(z, w);
        for (uint32_t j = b; j < e; ++j) {
            const uint2 v = in[j];
            lds_add(lt, tb, st, v.x, v.y);
        }
    }
    lds_flush(lt, tb, st);
}

// The stale churn of a multi-tile zone pass, after k_compact's tiles (which
// rewrote the zone's A-sides in place and placed the kept survivors):
//   * the stale window [lo, lo + m): the window source (wtmp, copied by k_body)
//     stored at its place and its pairs added — k_compact's window blocks;
//   * the stale tail [new_n, n): every old pair there destroyed — k_delta's tail
//     blocks — from the snapshot: a symbol rewritten as an A-side (hit at the
//     next position, hitmask) held `a`.
// Both in one workgroup's LDS table (a pair the tail drops and the window adds
// is one entry), dumped for k_zdr.
constexpr int CH_BT = 512;
constexpr int CH_U = 8;   // positions per thread per trip
template <typename S>
__global__ __launch_bounds__(CH_BT) void k_churn(DevState* zst, uint32_t round, S* __restrict__ cur,
                                                 S* __restrict__ oth, const uint32_t* __restrict__ hitmask,
                                                 const uint32_t* __restrict__ grpsum, const S* __restrict__ win,
                                                 Table tb, ZdrView zv, uint32_t wbase) {
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    __shared__ LdsTab<ZDR_N_CHURN> lt;
    __shared__ uint32_t s_surv[CH_BT / 64], s_left;
    DevState* st = zst;
    if (!merge_active(st, round)) return;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t n = st->n, new_n = st->new_n, m = st->m, mc = st->mc, a = st->a, b = st->b;
    const uint32_t pid_ab = (a << 16) | b;
    const uint32_t ntiles = (uint32_t)gbpe_div_up(n, TILE);
    lds_clear(lt);
    // window start = zone survivors - m (the group sums hold the survivors)
    {
        const uint32_t ngrp = (uint32_t)gbpe_div_up(ntiles, GRP);
        uint32_t sv = 0;
        for (uint32_t g = t; g < ngrp; g += CH_BT) sv += grpsum[g * GSTR];
        sv = wave_sum_u32(sv);
        if (lane == 0) s_surv[wid] = sv;
    }
    __syncthreads();
    uint32_t sv = 0;
    for (int w2 = 0; w2 < CH_BT / 64; ++w2) sv += s_surv[w2];
    const uint32_t lo = sv - m, woff = mc - m;
    const uint32_t G = gridDim.x, q = blockIdx.x;
    // this workgroup's window slice [w0, w1) and tail slice [t0, t1)
    const uint32_t wper = (m + G - 1) / G, w0 = lo + (q * wper < m ? q * wper : m),
                   w1 = lo + ((q + 1) * wper < m ? (q + 1) * wper : m);
    const uint32_t tlen = n > new_n ? n - new_n : 0u, tper = (tlen + G - 1) / G;
    const uint32_t t0 = new_n + (q * tper < tlen ? q * tper : tlen), t1 = new_n + ((q + 1) * tper < tlen ? (q + 1) * tper : tlen);
    if (w0 < w1 && wid == 0) {   // the symbol left of this slice: the survivor before the window, or the window itself
        uint32_t v = 0;
        if (w0 > lo) {
            v = win[woff + (w0 - lo) - 1];
        } else if (lo >= 1) {
            // the last survivor below new_n (k_compact's rule): last j < new_n with hit(j) == 0, A-side rewritten
            int64_t wi = (int64_t)(new_n - 1) / 32;
            uint32_t found = 0xFFFFFFFFu;
            while (wi >= 0 && found == 0xFFFFFFFFu) {
                const int64_t mywi = wi - lane;
                uint32_t inv = 0;
                if (mywi >= 0) inv = ~hitmask[mywi] & lane_mask32((uint64_t)mywi * 32, new_n);
                const unsigned long long has = __ballot(inv != 0u);
                if (has) {
                    const int l = __ffsll((long long)has) - 1;
                    const uint32_t inv_l = (uint32_t)__builtin_amdgcn_readlane(inv, l);
                    found = (uint32_t)((wi - l) * 32 + (31 - __clz(inv_l)));
                }
                wi -= 64;
            }
            if (found != 0xFFFFFFFFu) v = cur[found];   // (its in-place A-side rewrite, if any, is done)
        }
        if (lane == 0) s_left = v;
    }
    __syncthreads();
    // CH_U positions per thread per trip, all loaded before any LDS add: the slices
    // are long early (~2 mc / 256 symbols per workgroup at one workgroup per CU), and
    // one dependent load per position left every trip waiting on memory
    for (uint32_t d0 = w0 + t; d0 < w1; d0 += CH_BT * CH_U) {
        uint32_t x1[CH_U], x0[CH_U];
#pragma unroll
        for (int u = 0; u < CH_U; ++u) {
            const uint32_t d = d0 + (uint32_t)u * CH_BT;
            x1[u] = x0[u] = 0u;
            if (d < w1) {
                x1[u] = win[woff + (d - lo)];
                x0[u] = d == w0 ? s_left : (uint32_t)win[woff + (d - lo) - 1];
            }
        }
#pragma unroll
        for (int u = 0; u < CH_U; ++u) {
            const uint32_t d = d0 + (uint32_t)u * CH_BT;
            if (d >= w1 || d == 0) continue;
            oth[d] = (S)x1[u];
            const uint32_t u0 = x0[u] & TM, u1 = x1[u] & TM;
            if (!(x1[u] & WS) && u0 && u1) lds_add(lt, tb, st, (u0 << 16) | u1, 1u);
        }
    }
    for (uint32_t i0 = t0 + t; i0 < t1; i0 += CH_BT * CH_U) {
        uint32_t xi[CH_U], xp[CH_U], h1[CH_U], hp[CH_U];
#pragma unroll
        for (int u = 0; u < CH_U; ++u) {
            const uint32_t i = i0 + (uint32_t)u * CH_BT;
            xi[u] = xp[u] = h1[u] = hp[u] = 0u;
            if (i < t1 && i != 0) {
                xi[u] = cur[i];
                xp[u] = cur[i - 1];
                if (i + 1 < n) h1[u] = hitmask[(i + 1) / 32];
                hp[u] = hitmask[i / 32];
            }
        }
#pragma unroll
        for (int u = 0; u < CH_U; ++u) {
            const uint32_t i = i0 + (uint32_t)u * CH_BT;
            if (i >= t1 || i == 0) continue;
            // snapshot values: an A-side (hit at the next position) was rewritten to nw in place
            const uint32_t j1 = i + 1, jp = i;
            uint32_t x = xi[u], y = xp[u];
            if ((h1[u] >> (j1 % 32)) & 1u) x = a | (x & WS);   // (h1 = 0 past the zone's end)
            if ((hp[u] >> (jp % 32)) & 1u) y = a | (y & WS);
            if (x & WS) continue;
            const uint32_t tp = y & TM, ti = x & TM;
            if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
        }
    }
    lds_dump(lt, zv, wbase + q);
}

__global__ void k_clear_dirty_all(DevState* st, Table tb) {
    (void)st;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < tb.nblk) tb.dirty[i] = 1u;   // every block gets re-maxed
}

// dump live (count > 0) pairs
__global__ void k_dump_pairs(Table tb, uint32_t* pids, uint32_t* counts, uint32_t* nout, uint32_t cap) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > tb.mask) return;
    uint2 e = tb.slots[i];
    if (e.x && (int32_t)e.y > 0) {
        uint32_t k = atomicAdd(nout, 1u);
        if (k < cap) {
            pids[k] = e.x;
            counts[k] = e.y;
        }
    }
}

template <typename S>
__global__ void k_export_symbols(const S* __restrict__ s, uint32_t* __restrict__ out, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = s[i];
    out[i] = (x & Sym<S>::TM) | ((x & Sym<S>::WS) ? 0x10000u : 0u);
}

// the inverse: reference u32 layout (bit16 = word start) -> S (consolidation)
template <typename S>
__global__ void k_import_symbols(const uint32_t* __restrict__ in, S* __restrict__ s, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = in[i];
    s[i] = (S)((x & Sym<S>::TM) | ((x & 0x10000u) ? Sym<S>::WS : 0u));
}

}  // namespace

// the sector-sparse merge loop: sparse.h
#include "sparse.h"
