// BPE training merge loop on MI355X (gfx950).
//
// Replaces the reference's 8-dispatch-per-merge WGSL pipeline
// (training-pipeline.js:178-222: clear_table → pair_count_b → find_max_pair4 →
// find_max_pair_final_det → setup_merge → merge_reduce_b → scan_blocks →
// finalize_compact_b, train.wgsl) with an incremental design:
//
//   * the pair-count table PERSISTS across merges; instead of clearing 2^21
//     slots and recounting every pair of the stream each merge
//     (train.wgsl:188-202, 366-431), a merge only emits count deltas at its
//     merge sites, aggregated per workgroup in LDS, then added into the
//     global table — exact counts, no silent drops (train.wgsl:422-429);
//   * argmax is a two-level tournament: per-2048-slot block maxima, only
//     recomputed for blocks a merge touched, then one workgroup reduces them
//     with the reference's tie-break (higher count, then smaller a<<16|b,
//     train.wgsl:83-85);
//   * the stream pass is two streaming kernels over 8192-symbol tiles:
//     k_delta (reads the stream; writes a 1-bit merge-site mask, per-tile
//     survivor counts and count deltas) and k_compact (reads stream + mask,
//     rewrites merged symbols in place, scatters survivors into the
//     ping-pong buffer at a two-level tile prefix).  k_compact never reads a
//     neighbour symbol, so snapshot semantics (train.wgsl:476) hold without
//     the reference's race;
//   * symbols are u16 (bit 15 = word start) whenever every token id fits in
//     15 bits (vocab <= 32768), else u32 with bit 16 (train.wgsl:36-37), so
//     the common 32K-vocab case moves half the bytes.
//
// The reference's compaction quirk (bpe_finalize_compact_b bounded by the
// NEW symbol count, train.wgsl:605-607 + 698/727) is reproduced by default:
// survivors whose old index is >= the new count are not scattered and the
// stale ping-pong contents stay in the stream; k_compact's tail blocks add
// the pairs of that stale window to the count table.
//
// Per merge: k_select (1 WG) → k_delta → k_compact (tiles + tail) → k_refresh.

#include "common.h"
#include "scan.h"

#include <algorithm>
#include <chrono>
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
    // ── sharded training (gbpe_shard_*); n / new_n above are then LOCAL: the
    //    local stream length and the local keep limit ──
    uint32_t sharded, rank, world, stall;
    uint32_t dused;        // occupied slots of the per-merge delta table
    uint32_t dcount;       // delta entries of this merge (the record's list length)
    uint32_t need_l, need_w;   // capacities a stalled merge asked for (max over ranks)
    uint32_t owner;        // rank that appended this merge's stale window
    uint32_t nl_next;      // local length after this merge
    uint32_t m_glob;       // global stale-window length of this merge
    uint32_t pln;          // local length of the previous input stream (stale-window source)
    uint64_t gn;           // global stream length
    uint64_t off;          // global offset of the local stream
    uint64_t poff;         // global offset of the previous input stream
    uint64_t off_next;
    uint64_t gnew;         // gn - mc
    uint32_t peak_l, peak_w;   // largest record list / window piece of this step (capacity sizing)
    uint32_t dfull;            // the delta table overflowed this merge
    // ── sector-sparse loop (n / new_n above stay GLOBAL; the zone has its own DevState) ──
    uint32_t B;            // body length: symbols in the word-aligned sectors before the zone
    uint32_t Bp;           // body length during the previous merge (stale-window source offset)
    uint32_t body_rm;      // B-sides removed from the body by this merge
    uint32_t sp_abort;     // a selected merge does not fit the zone: not run, host goes dense
    uint32_t sel_round;    // sector-sparse: round + 1 of the merge k_body selected
    uint64_t sp_bytes;     // sector-sparse: bytes moved by the multi-tile zone passes (k_refresh adds them)
    uint32_t zlast;        // sector-sparse: zone length of the rank that holds the zone (global knowledge)
    uint32_t ln_last;      // sharded: the last rank's local length after the last merge (from the records)
    uint32_t is_last;      // sector-sparse: this rank holds the zone (single GPU: always)
    uint32_t cand;         // candidate sectors of this merge (trace)
    uint32_t hitsec;       // sectors with a site (trace)
    uint32_t mc_prev;      // sector-sparse, single GPU: the last merge's count (k_refresh), for the zone rule
                           // (never written by a commit: a reader beside k_body would see it unchanged)
    uint32_t enter_lim;    // dense loop: end the step at the first merge whose count is <= this (the host
                           // can then enter the sector-sparse loop; 0 = off)
};
static_assert(sizeof(DevState) <= 256, "state");

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
#define TKT(i) kt_put(r, 1u, (i), wall_clock64())   // k_tail's own phases (workgroup slot 1)
#define TKTV(i, v) kt_put(r, 1u, (i), (v))
#else
#define TKT(i) ((void)0)
#define TKTV(i, v) ((void)0)
#define KT(i) ((void)0)
#define KTV(i, v) ((void)0)
#define KTR(i) ((void)0)
#endif

// exchange-record header words of sharded training (gpubpe/sharded.py mirrors them)
enum : uint32_t {
    H_ACTIVE = 0, H_L, H_KEPT, H_M, H_W, H_LASTSYM, H_HASLAST, H_SURV, H_LN, H_MC, H_A, H_B, H_ID, H_DFULL,
    H_ZN = 14,             // sector-sparse records: the zone length after the merge (last rank), its window m
    H_ZM = 15, HDR = 16
};

enum : uint32_t {
    ERR_TABLE_FULL = 1, ERR_COUNT_MISMATCH = 2, ERR_PAIR_MISSING = 4, ERR_SPIN = 8,
    ERR_SHARD_CAPACITY = 16,   // a rank's stream outgrew its buffers (stale window appended)
    ERR_SHARD_RECORD = 32,     // exchange records disagree (ranks out of step)
    ERR_SHARD_LAYOUT = 64,     // gathered survivor / length totals do not add up
    ERR_SPARSE_WINDOW = 128    // sector-sparse: a stale window reaches past the zone's stale buffer
};

struct Table {
    uint2* slots;      // .x = pid (0 = empty), .y = count (u32, wraps for transient negatives)
    uint32_t mask;     // slots - 1
    uint64_t* bmax;    // per block: (count << 32) | ~pid, 0 when empty
    uint32_t* dirty;   // per block flag
    uint32_t* dlist;   // dirty block list
    uint32_t* blive;   // per block: entries with count > 0
    uint32_t nblk;
    uint32_t* used;    // occupied-slot counter (DevState::used or ::dused)
    uint32_t* full;    // non-null: a full table sets *full instead of the fatal error (delta table)
};

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
    if (tb.full) *tb.full = 1u;   // per-merge delta table sized too small: the merge stalls and retries bigger
    else atomicOr(&st->err, ERR_TABLE_FULL);
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

template <int N>
__device__ __forceinline__ void lds_add(LdsTab<N>& t, const Table& tb, DevState* st, uint32_t pid, uint32_t d) {
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

// Up to 8 (pid, delta) adds with their home-slot key loads issued together: at
// the table's low load factor nearly every live pair sits in its home slot, so
// a batch costs one round trip instead of one per entry; the rest (new keys,
// collisions) take the full probe.  Entries with pid or delta 0 are skipped.
__device__ __forceinline__ void table_add8(const Table& tb, DevState* st, const uint32_t (&kk)[8],
                                           const uint32_t (&vv)[8]) {
    uint32_t hs[8], hk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hs[j] = (kk[j] && vv[j]) ? (gbpe_fmix32(kk[j]) & tb.mask) : 0u;
        hk[j] = __hip_atomic_load(&tb.slots[hs[j]].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
template <int N>
__device__ __forceinline__ void lds_flush(LdsTab<N>& t, const Table& tb, DevState* st) {
    __syncthreads();
    const uint32_t nt = blockDim.x;
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

__device__ void select_merge(DevState* st, Table tb, uint32_t* __restrict__ log, uint32_t* __restrict__ grpsum,
                             uint32_t* __restrict__ nlog, uint32_t* __restrict__ rec, DevState* zst, uint32_t exact);

// (unused launch argument: the selection fused into k_refresh was measured slower)
struct FusedSel {
    uint32_t* log = nullptr;
    uint32_t* grpsum = nullptr;
    uint32_t exact = 0;
};

// recompute block maxima for dirty blocks; with `finish`, also closes the
// merge of `round` (state.symbol_count := new count, train.wgsl:605-607)
template <typename S>
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
        if (threadIdx.x < NW) s_g.w[threadIdx.x] = reinterpret_cast<const uint32_t*>(st)[threadIdx.x];
        else if (zst && threadIdx.x < 2 * NW) s_z.w[threadIdx.x - NW] = reinterpret_cast<const uint32_t*>(zst)[threadIdx.x - NW];
        __syncthreads();
        const DevState& g = s_g.d;
        const DevState& z = s_z.d;
        const bool fin = finish == 2 ? (!g.stop && !g.sp_abort && g.sel_round == round + 1u)
                                     : (!g.stop && !g.stall && g.merges_done == round + 1u);
        if (fin && threadIdx.x == 0) {
            if (zst) {   // sector-sparse: global length, body length, zone length
                if (finish == 2) {
                    st->merges_done = round + 1u;
                    st->next_id = g.next_id + 1u;
                    st->epoch = g.epoch + 1u;
                    st->mc_prev = g.mc;
                }
                if (clog) {
                    clog[2 * round] = g.cand;
                    clog[2 * round + 1] = g.hitsec;
                }
                st->cand = 0u;
                st->hitsec = 0u;
                st->tail_total = g.tail_total + z.m;
                const uint32_t n = g.new_n, B = g.B - g.body_rm, zn = n - B;
                st->n = n;
                st->Bp = g.B;
                st->B = B;
                st->body_rm = 0u;
                zst->n = zn;
                if (!g.sharded) st->zlast = zn;   // sharded: from the records (k_shard_apply)
                if (!z.valid_total && g.is_last)   // multi-tile zone: k_delta + k_compact stream it twice, plus the window copy
                    st->sp_bytes = g.sp_bytes + (uint64_t)sizeof(S) * (2ull * z.n + zn + 2ull * g.mc);
                if (z.valid_total && z.valid_total != zn + 1u) atomicOr(&st->err, ERR_COUNT_MISMATCH);
            } else if (g.sharded) {   // commit the new global layout computed by k_shard_recv
                st->tail_total = g.tail_total + g.m_glob;
                st->poff = g.off;
                st->pln = g.n;
                st->n = g.nl_next;
                st->off = g.off_next;
                st->gn = g.gnew;
            } else {
                st->tail_total = g.tail_total + g.m;
                st->n = g.new_n;
            }
        }
    }
    // this WG's contiguous run of blocks (<= 64): all flags (and, for `part`, the
    // maxima kept from before) in one load; then every wave re-maxes its share of
    // the dirty ones, one 256-slot block at a time (no workgroup barrier per block:
    // a merge dirties a few blocks per workgroup, each holding a few live pairs)
    __shared__ uint64_t s_dmask;
    __shared__ uint64_t s_bm[64];
    const uint32_t per = (tb.nblk + gridDim.x - 1) / gridDim.x;   // <= 64 (host-sized grid)
    const uint32_t b0 = blockIdx.x * per;
    if (threadIdx.x < 64) {
        const uint32_t blk = b0 + threadIdx.x;
        const bool in = threadIdx.x < per && blk < tb.nblk;
        if (part) s_bm[threadIdx.x] = in ? tb.bmax[blk] : 0ull;
        const bool d = in && tb.dirty[blk];
        const unsigned long long m = __ballot(d);
        if (threadIdx.x == 0) s_dmask = m;
    }
    __syncthreads();
    {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        constexpr int NV = (1 << BLK_LOG2) / 2 / 64;   // 16-byte loads per lane
        uint64_t dm = s_dmask;
        for (int k = 0; dm; ++k) {   // (wave-uniform)
            const uint32_t bit = (uint32_t)(__ffsll((long long)dm) - 1);
            dm &= dm - 1;
            if ((k & (TPB / 64 - 1)) != wid) continue;
            const uint32_t blk = b0 + bit;
            const uint4* sl = reinterpret_cast<const uint4*>(tb.slots + ((uint64_t)blk << BLK_LOG2));
            uint4 e[NV];
#pragma unroll
            for (int q = 0; q < NV; ++q) e[q] = sl[lane + q * 64];
            uint64_t best = 0;
            uint32_t live = 0;
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                if (e[q].x && (int32_t)e[q].y > 0) {
                    const uint64_t key = ((uint64_t)e[q].y << 32) | (uint32_t)(~e[q].x);
                    best = key > best ? key : best;
                    ++live;
                }
                if (e[q].z && (int32_t)e[q].w > 0) {
                    const uint64_t key = ((uint64_t)e[q].w << 32) | (uint32_t)(~e[q].z);
                    best = key > best ? key : best;
                    ++live;
                }
            }
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t o = __shfl_xor(best, off);
                best = o > best ? o : best;
                live += __shfl_xor(live, off);
            }
            if (lane == 0) {
                tb.bmax[blk] = best;
                tb.blive[blk] = live;
                tb.dirty[blk] = 0u;
                s_bm[bit] = best;
            }
        }
    }
    __syncthreads();
    if (part && threadIdx.x < 64) {   // this workgroup's maximum, for sel_inline
        uint64_t best = s_bm[threadIdx.x];
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(best, off);
            best = o > best ? o : best;
        }
        if (threadIdx.x == 0) {
            part[blockIdx.x] = best;
            if (finish == 2) KTR(5);
        }
    }
}

constexpr uint32_t GRP = 64;    // tiles per group sum (two-level tile prefix)
constexpr uint32_t GSTR = 64;   // group sums 256 B apart: each is its own atomic serialisation point

// argmax over block maxima + the reference's bpe_setup_merge (train.wgsl:340-364),
// by one workgroup of any size <= SEL_THREADS
__device__ void select_merge(DevState* st, Table tb, uint32_t* __restrict__ log, uint32_t* __restrict__ grpsum,
                             uint32_t* __restrict__ nlog, uint32_t* __restrict__ rec, DevState* zst, uint32_t exact) {
    __shared__ uint64_t red[SEL_THREADS / 64];
    __shared__ uint32_t rlive[SEL_THREADS / 64];
    const uint32_t nt = blockDim.x;
    if (rec && threadIdx.x == 0) rec[H_L] = 0u;   // the send kernel's list blocks add their counts into it
    if (st->stop || st->stall || st->sp_abort) return;
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
    for (int off = 32; off > 0; off >>= 1) {
        uint64_t o = __shfl_xor(best, off);
        best = o > best ? o : best;
        live += __shfl_xor(live, off);
    }
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
    st->dcount = 0u;
    st->dused = 0u;
    st->dfull = 0u;
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
        if ((uint64_t)st->n < 2ull * mc + st->Bp) {   // cannot happen after the check below held
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
    if (st->sharded) {   // global new length; the local keep limit (train.wgsl:727 on the global stream)
        const uint64_t gnew = st->gn - mc;
        st->gnew = gnew;
        uint64_t lim = st->n;
        if (!(st->sharded & 2u)) lim = gnew > st->off ? (gnew - st->off < st->n ? gnew - st->off : st->n) : 0u;
        st->new_n = (uint32_t)lim;
    } else {
        st->new_n = st->n - mc;
    }
    if (nlog) nlog[d] = st->n;
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
                                                        uint32_t* __restrict__ grpsum, uint32_t* __restrict__ nlog,
                                                        uint32_t* __restrict__ rec, DevState* zst, uint32_t exact) {
    select_merge(st, tb, log, grpsum, nlog, rec, zst, exact);
}

// the next merge's count (the table maximum): the sparse entry decision before any merge ran
__global__ __launch_bounds__(1024) void k_topcount(Table tb, uint32_t* __restrict__ out) {
    __shared__ uint64_t red[16];
    uint64_t best = 0;
    for (uint32_t i = threadIdx.x; i < tb.nblk; i += 1024) {
        const uint64_t v = tb.bmax[i];
        best = v > best ? v : best;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
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
    for (int off = 32; off > 0; off >>= 1) live += __shfl_xor(live, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) live += red[w];
        st->live = live;
        if (live > st->max_live) st->max_live = live;
    }
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
                                               uint32_t ngroups = 0xFFFFFFFFu) {
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
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
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
        lds_flush(lt, tb, st);
        for (int off = 32; off > 0; off >>= 1) tail += __shfl_xor(tail, off);
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
                                                  uint32_t* __restrict__ grpsum, uint32_t eager_tiles, uint32_t ngroups) {
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
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
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
    lds_flush(lt, tb, st);
    for (int off = 32; off > 0; off >>= 1) tail += __shfl_xor(tail, off);
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
                                                 const S* __restrict__ win = nullptr, const DevState* gst = nullptr) {
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
    if (tl >= ntiles) {
        if (EXACT || st->sharded) return;   // sharded: the window is handled by k_shard_recv
        // ── stale tail window ──
        const uint32_t m = st->m;
        if (m == 0) return;
        LdsTab<LTAB>& lt = *reinterpret_cast<LdsTab<LTAB>*>(arena);
        __shared__ uint32_t left_val;
        lds_clear(lt);
        uint32_t lo = new_n - m;
        const uint32_t tb0 = tl - ntiles, ntb = gridDim.x - ntiles;
        uint32_t woff = 0;
        if (ZONE) {   // window start = zone survivors - m (the group sums hold the survivors)
            __shared__ uint32_t s_surv[CTPB / 64];
            const uint32_t ngrp = (uint32_t)gbpe_div_up(ntiles, GRP);
            uint32_t sv = 0;
            for (uint32_t g = t; g < ngrp; g += CTPB) sv += grpsum[g * GSTR];
            for (int off = 32; off > 0; off >>= 1) sv += __shfl_xor(sv, off);
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
                    const uint32_t inv_l = __shfl(inv, l);
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
    uint32_t incl = cnt;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
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
    if (tl == ntiles - 1 && t == 0 && !st->sharded &&
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

// ─── sector-sparse merge loop ──────────────────────────────────
//
// Late in training a merge's count is a tiny fraction of the stream, yet the
// dense pass above reads the whole stream twice per merge.  The sparse loop
// re-lays the stream out as
//   * a BODY of word-aligned sectors: sector k starts at the first word start at
//     or after k*SEC and keeps its symbols compacted at its own start.  Pairs
//     never cross a word start (train.wgsl:395, 483, 493), so sectors merge
//     independently and their first symbol is never a B-side;
//   * a token-presence bitmap (row = token id, bit = sector): a merge (a, b) can
//     only have sites in sectors whose a-row and b-row bits are both set.  Bits
//     are set when a token appears in a sector and never cleared (a superset);
//   * a dense ZONE: the last >= 5*mc symbols, run by the dense kernels on their
//     own ping-pong buffers.  It carries the reference's compaction quirk (the
//     stale window always lands at the end of the stream).  Its coordinates are
//     global position - B (body length), which shifts as the body loses
//     symbols, so the stale window is copied out (k_body's copy blocks) instead
//     of being left in place.
// Per merge: k_select → k_body (candidate sectors + window copy) → k_delta (zone)
// → k_compact<ZONE> → k_refresh.
constexpr uint32_t SP_WPW_MIN = 16;  // fewest bitmap words per k_body workgroup (sizes its byte counters)
constexpr uint32_t SP_CH = 256;      // symbols per wave pass over a sector (4 per lane)
constexpr uint32_t SP_INV = 0xFFFFFFFFu;
constexpr uint32_t SP_SHRINKS = 64;  // zone shrinks per sparse entry (sector capacity)

// Per-sector pair signature: a 1024-bit Bloom filter (2 hash bits) of every pair
// the sector has held since the filters were last rebuilt.  The token bitmap
// gives candidate sectors; the signature drops most of those where a and b are
// both present but never adjacent.
constexpr uint32_t SP_SIGW = 32;     // u32 words per sector signature
__device__ __forceinline__ uint32_t sig_hash(uint32_t pid) { return gbpe_fmix32(pid ^ 0x9E3779B9u); }
__device__ __forceinline__ bool sig_has(const uint32_t* __restrict__ sig, uint32_t pid) {
    const uint32_t h = sig_hash(pid), b1 = h & 1023u, b2 = (h >> 16) & 1023u;
    return ((sig[b1 >> 5] >> (b1 & 31u)) & (sig[b2 >> 5] >> (b2 & 31u)) & 1u) != 0u;
}
// global signature (k_body): no-return atomics, no test load on the merge's critical path
__device__ __forceinline__ void sig_or(uint32_t* __restrict__ sig, uint32_t pid) {
    const uint32_t h = sig_hash(pid), b1 = h & 1023u, b2 = (h >> 16) & 1023u;
    atomicOr(&sig[b1 >> 5], 1u << (b1 & 31u));
    atomicOr(&sig[b2 >> 5], 1u << (b2 & 31u));
}
// LDS signature (k_sp_bits): test first, most bits are already set
__device__ __forceinline__ void sig_set(uint32_t* __restrict__ sig, uint32_t pid) {
    const uint32_t h = sig_hash(pid), b1 = h & 1023u, b2 = (h >> 16) & 1023u;
    const uint32_t m1 = 1u << (b1 & 31u), m2 = 1u << (b2 & 31u);
    if (!(sig[b1 >> 5] & m1)) atomicOr(&sig[b1 >> 5], m1);
    if (!(sig[b2 >> 5] & m2)) atomicOr(&sig[b2 >> 5], m2);
}

// a sector's first wave pass: 4 symbols per lane and the one after the pass
// (+ their word multiplicities in the lexicon body, else 1)
template <typename S>
__device__ __forceinline__ void sector_first(const S* __restrict__ p, const uint32_t* __restrict__ mp, uint32_t cnt,
                                             uint32_t (&f)[5], uint32_t (&fm)[4]) {
    const uint32_t i0 = 4u * (uint32_t)(threadIdx.x & 63);
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = (i0 + k < cnt) ? (uint32_t)p[i0 + k] : 0u;
    f[4] = (SP_CH < cnt) ? (uint32_t)p[SP_CH] : 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) fm[k] = mp ? ((i0 + k < cnt) ? mp[i0 + k] : 0u) : 1u;
}

// One wave merges one sector in place (snapshot semantics, k_delta's delta rule,
// survivors compacted to the sector's front).  In the lexicon body (mp != null)
// every symbol carries its word's multiplicity, which weights its count deltas
// and moves with it.  Returns the B-sides removed (weighted: stream symbols).
template <typename S, int NT = LTAB_T>
__device__ uint32_t body_sector(S* __restrict__ p, uint32_t* __restrict__ mp, uint32_t cnt, uint32_t a, uint32_t b,
                                uint32_t nw, LdsTab<NT>& lt, const Table& tb, DevState* st, uint32_t* __restrict__ sig,
                                uint32_t& out_cnt, const uint32_t (&first)[5], const uint32_t (&firstm)[4]) {
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    const int lane = threadIdx.x & 63;
    const uint32_t pid_ab = (a << 16) | b;
    uint32_t c1 = 0, c2 = 0, out = 0, removed = 0;
    for (uint32_t c0 = 0; c0 < cnt; c0 += SP_CH) {
        const uint32_t i0 = c0 + 4u * lane;
        // X[0..1] = the two symbols before this lane's four, X[6] = the one after
        uint32_t X[7], nx, M[4];
        if (c0 == 0) {   // the first pass's symbols were loaded by the caller (sector_first)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                X[2 + k] = first[k];
                M[k] = firstm[k];
            }
            nx = first[4];
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) X[2 + k] = (i0 + k < cnt) ? (uint32_t)p[i0 + k] : 0u;
            nx = (c0 + SP_CH < cnt) ? (uint32_t)p[c0 + SP_CH] : 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k) M[k] = mp ? ((i0 + k < cnt) ? mp[i0 + k] : 0u) : 1u;
        }
        uint32_t pm1 = __shfl_up(X[5], 1), pm2 = __shfl_up(X[4], 1);
        uint32_t np = __shfl_down(X[2], 1);
        if (lane == 0) {
            pm1 = c1;
            pm2 = c2;
        }
        if (lane == 63) np = nx;
        X[0] = pm2;
        X[1] = pm1;
        X[6] = np;
        c1 = __shfl(X[5], 63);
        c2 = __shfl(X[4], 63);
        // h[j] = hit at the position of X[j]: a B-side (no word-start bit) after an a
        bool h[7];
        h[0] = false;
#pragma unroll
        for (int j = 1; j < 7; ++j) h[j] = X[j] == b && (X[j - 1] & TM) == a;
        uint32_t keep = 0, vals[4];
        bool touched = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = k + 2;
            const bool valid = i0 + k < cnt;
            const uint32_t w = M[k];   // a pair's occurrences = its right symbol's word multiplicity
            if (valid && !h[j]) keep |= 1u << k;
            if (valid && h[j]) removed += w;
            vals[k] = h[j + 1] ? (nw | (X[j] & WS)) : X[j];
            touched |= valid && (h[j] || h[j + 1]);
            if (valid && !(X[j] & WS) && (h[j - 1] || h[j] || h[j + 1])) {
                const uint32_t tp = X[j - 1] & TM, ti = X[j] & TM;
                if (tp && ti) {
                    const uint32_t pid = (tp << 16) | ti;
                    if (pid != pid_ab) lds_add(lt, tb, st, pid, 0u - w);   // old pair destroyed
                }
                if (!h[j]) {
                    if (h[j - 1]) {
                        const uint32_t t2 = h[j + 1] ? nw : ti;
                        if (t2) {
                            lds_add(lt, tb, st, (nw << 16) | t2, w);
                            sig_or(sig, (nw << 16) | t2);
                        }
                    } else if (h[j + 1] && tp) {
                        lds_add(lt, tb, st, (tp << 16) | nw, w);
                        sig_or(sig, (tp << 16) | nw);
                    }
                }
            }
        }
        const uint32_t kc = __popc(keep);
        uint32_t incl = kc;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off);
            if (lane >= off) incl += o;
        }
        const uint32_t tot = __shfl(incl, 63);
        // every read of this pass happened above; writes land at or before their source
        if (out != c0 || __any(touched)) {
            uint32_t w = out + incl - kc;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((keep >> k) & 1u) {
                    if (mp) mp[w] = M[k];
                    p[w++] = (S)vals[k];
                }
        }
        out += tot;
    }
    out_cnt = out;
    for (int off = 32; off > 0; off >>= 1) removed += __shfl_xor(removed, off);   // per lane → the wave's
    return removed;
}

// Single-workgroup zone pass (zone <= ZMAX symbols): k_delta + k_compact<ZONE>
// in one workgroup.  Each thread holds 32 consecutive zone symbols in registers
// and builds k_delta's branch-free site masks; only positions next to a site or
// in the stale tail touch the LDS copy and the delta table.  Kept survivors
// (A-sides rewritten, also in place: the reference's ping buffer) are compacted
// into the other zone buffer and the stale window follows them.  The window
// source is read from the other buffer before anything is written to it.
// k_body runs as 1024-thread workgroups (16 waves: more sectors in flight, a
// zone up to 32K symbols in one workgroup) while the zone is large, and as
// 256-thread ones late in training (small zone, lower latency per launch).
template <typename S, int BT> struct ZoneDim {
    static constexpr int ZPT = (BT == 1024 && sizeof(S) == 4) ? 16 : 32;   // zone positions per thread
    static constexpr uint32_t ZMAX = (uint32_t)BT * ZPT;   // 8192 (256) / 32768 or 16384 (1024) symbols
    static constexpr uint32_t ZWIN = ZMAX / 3 + 64;         // >= mc: the zone holds >= 3 mc (sel_inline's rule)
};
template <typename S, int BT>
struct ZoneLds {
    uint4 xv[ZoneDim<S, BT>::ZMAX * sizeof(S) / 16];   // the zone (symbol i = ((S*)xv)[i])
    S wb[ZoneDim<S, BT>::ZWIN];
    uint32_t wsum[BT / 64], wtail[BT / 64];
    S trash[64];   // the zone pass's unconditional stores of dropped symbols
};

__device__ __forceinline__ uint32_t lane_mask_n(uint64_t i0, uint64_t lim, int n) {
    // bits k with i0 + k < lim, k < n (n <= 32)
    const uint32_t full = n == 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    return i0 >= lim ? 0u : (i0 + n <= lim ? full : ((1u << (uint32_t)(lim - i0)) - 1u));
}

// zout (the persistent tail loop, k_tail): the delta table is shared with the body
// pass (neither cleared nor flushed here) and m, the new zone length go to zout[0..1]
template <typename S, bool EXACT, int BT, int NT = LTAB_T, int ZPT_ = ZoneDim<S, BT>::ZPT>
__device__ void zone_one(DevState* st, DevState* zst, const DevState& gs, const DevState& zs, S* __restrict__ zc,
                         S* __restrict__ zo, ZoneLds<S, BT>& L,
                         LdsTab<NT>& lt, const Table& tb, uint32_t a, uint32_t b, uint32_t nw, uint32_t mc,
                         uint64_t* __restrict__ bytes, uint32_t round, uint32_t* zout = nullptr) {
    (void)round;   // phase stamps only (-DGBPE_KTRACE)
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    constexpr int ZPT = ZPT_;                // zone positions per thread (<= ZoneDim's: the LDS is sized for that)
    static_assert(ZPT <= ZoneDim<S, BT>::ZPT && ZPT * sizeof(S) % 16 == 0, "zone positions per thread");
    constexpr int V = ZPT * sizeof(S) / 16;  // 16-byte vectors per thread
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t z = zs.n;   // launch snapshots (LDS): no state round trip before the zone loads
    const uint32_t lim = EXACT ? z : z - mc;
    const uint32_t pid_ab = (a << 16) | b;
    const uint32_t i0 = (uint32_t)t * ZPT;
    S* xs = reinterpret_cast<S*>(L.xv);
    uint32_t x[ZPT];
    {
        uint4 v[V];
        const uint4* src = reinterpret_cast<const uint4*>(zc + i0);   // zone buffers hold >= 2 tiles
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = src[k];
#pragma unroll
        for (int k = 0; k < V; ++k) L.xv[t * V + k] = v[k];
        const S* e = reinterpret_cast<const S*>(v);
#pragma unroll
        for (int k = 0; k < ZPT; ++k) x[k] = i0 + k < z ? (uint32_t)e[k] : 0u;
    }
    if (!EXACT) {   // window source: global n - 2mc in the previous stream (sharded: it began at poff, now off)
        const uint64_t src0 = (uint64_t)gs.n + gs.off - gs.poff - 2ull * mc - gs.Bp;
        for (uint32_t u = t; u < mc; u += BT) L.wb[u] = zo[src0 + u];
    }
    if (!zout) lds_clear(lt);
    __syncthreads();
    if (t == 0) KT(2);
    const uint32_t xm2 = i0 >= 2 ? (uint32_t)xs[i0 - 2] : 0u, xm1 = i0 >= 1 ? (uint32_t)xs[i0 - 1] : 0u;
    const uint32_t nxr = i0 + ZPT < z ? (uint32_t)xs[i0 + ZPT] : 0u;
    uint32_t eb = 0, ea = 0;
#pragma unroll
    for (int k = 0; k < ZPT; ++k) {
        eb |= (x[k] == b ? 1u : 0u) << k;
        ea |= ((x[k] & TM) == a ? 1u : 0u) << k;
    }
    const uint32_t inb = lane_mask_n(i0, z, ZPT);
    const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a ? 1u : 0u)) & inb;
    const uint32_t h_m1 = (i0 >= 1 && i0 - 1 < z && xm1 == b && (xm2 & TM) == a) ? 1u : 0u;
    const uint32_t h_32 = (nxr == b && (ea >> (ZPT - 1))) ? 1u : 0u;
    const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_32 << (ZPT + 1));
    const uint32_t below = lane_mask_n(i0, lim, ZPT);
    const uint32_t surv = inb & ~hitm, keep = surv & below;
    const uint32_t rwm = ((hitm >> 1) | (h_32 << (ZPT - 1))) & inb;
    uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
    for (uint32_t i = (lim > 1u ? lim : 1u) + t; i < z; i += BT) {   // stale tail: old pairs destroyed
        const uint32_t xi = xs[i];
        if (xi & WS) continue;
        const uint32_t tp = xs[i - 1] & TM, ti = xi & TM;
        if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
    }
    while (rel) {
        const int k = __ffs(rel) - 1;
        rel &= rel - 1;
        const uint32_t i = i0 + k;
        if (i == 0) continue;
        const uint32_t xi = xs[i];
        if (xi & WS) continue;
        const uint32_t xp = xs[i - 1];
        const bool hm = (hbits >> k) & 1u, h0 = (hbits >> (k + 1)) & 1u, hp = (hbits >> (k + 2)) & 1u;
        const uint32_t tp = xp & TM, ti = xi & TM;
        if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
        if (!h0) {
            if (hm) {
                const uint32_t t2 = hp ? nw : ti;
                if (t2) lds_add(lt, tb, st, (nw << 16) | t2, 1u);
            } else if (hp && tp) {
                lds_add(lt, tb, st, (tp << 16) | nw, 1u);
            }
        }
    }
    if (t == 0) KT(3);
    // block exclusive scan of the kept counts; tail survivors sum to m
    const uint32_t kc = __popc(keep);
    uint32_t incl = kc, tl = __popc(surv & ~below);
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    for (int off = 32; off > 0; off >>= 1) tl += __shfl_xor(tl, off);
    if (lane == 63) L.wsum[wid] = incl;
    if (lane == 0) L.wtail[wid] = tl;
    __syncthreads();
    if (t == 0) KT(7);
    uint32_t pre = incl - kc, Kz = 0, m = 0;
#pragma unroll
    for (int w2 = 0; w2 < BT / 64; ++w2) {
        pre += w2 < wid ? L.wsum[w2] : 0u;
        Kz += L.wsum[w2];
        m += L.wtail[w2];
    }
    // The new zone is assembled in LDS over the old copy (every read of it is
    // done) and leaves in whole 16-byte stores: per-symbol global stores at a
    // lane stride of ZPT symbols cost a cache line per lane and instruction.
    // In LDS the 16-byte chunks are XOR-swizzled within groups of 8: lanes
    // write ZPT symbols apart, which unswizzled lands every lane of a wave on
    // the same two banks.
    constexpr uint32_t PV = 16 / sizeof(S), PVL = sizeof(S) == 2 ? 3 : 2;
    auto swz = [](uint32_t o) -> uint32_t {
        const uint32_t c = o >> PVL;
        return ((c ^ ((c >> 3) & 7u)) << PVL) | (o & (PV - 1u));
    };
    // branch-free: every position stores (dropped ones into a per-lane trash
    // slot); the A-side rewrites of the reference's in-place ping buffer are
    // the only global stores, one per rewritten position
    uint32_t wsm = 0;
#pragma unroll
    for (int k = 0; k < ZPT; ++k) {
        const bool rw = (rwm >> k) & 1u;
        const uint32_t v = rw ? (nw | (x[k] & WS)) : x[k];
        wsm |= ((x[k] & WS) ? 1u : 0u) << k;
        const uint32_t o = pre + (uint32_t)__popc(keep & ((1u << k) - 1u));
        S* dst = ((keep >> k) & 1u) ? &xs[swz(o)] : &L.trash[lane];
        *dst = (S)v;
    }
    for (uint32_t r = rwm; r; r &= r - 1) {
        const int k = __ffs(r) - 1;
        zc[i0 + k] = (S)(nw | (((wsm >> k) & 1u) ? WS : 0u));
    }
    if (t == 0) KT(8);
    if (!EXACT && m) {
        __syncthreads();
        const uint32_t woff = mc - m;
        for (uint32_t j = t; j < m; j += BT) {
            const uint32_t x1 = L.wb[woff + j];
            // left of the window: the last kept survivor (Kz > 0: the zone holds >= 5 mc)
            const uint32_t x0 = j ? (uint32_t)L.wb[woff + j - 1] : (Kz ? (uint32_t)xs[swz(Kz - 1)] : 0u);
            xs[swz(Kz + j)] = (S)x1;
            if (!(x1 & WS) && (x0 & TM) && (x1 & TM)) lds_add(lt, tb, st, ((x0 & TM) << 16) | (x1 & TM), 1u);
        }
    }
    __syncthreads();
    if (t == 0) KT(9);
    {
        const uint32_t tot = Kz + m, nfull = tot / PV;
        uint4* dst = reinterpret_cast<uint4*>(zo);
        for (uint32_t q = t; q < nfull; q += BT) dst[q] = L.xv[q ^ ((q >> 3) & 7u)];
        for (uint32_t j = nfull * PV + t; j < tot; j += BT) zo[j] = xs[swz(j)];
    }
    if (t == 0) KT(4);
    if (!zout) lds_flush(lt, tb, st);
    if (t == 0) {
        if (zout) {
            zout[0] = m;
            zout[1] = Kz + m;
        } else {
            zst->m = m;
            zst->valid_total = Kz + m + 1u;   // survivors + 1 (k_refresh checks it against the new layout)
        }
        // zone read, window source read, kept survivors + window written
        atomicAdd(bytes, (uint64_t)sizeof(S) * ((uint64_t)z + (EXACT ? 0u : mc) + Kz + m));
    }
}

// ── segmented zone pass (zones of 32K-1M symbols) ──
// A zone too large for one workgroup but far smaller than the stream (merges
// ~500-8000 at 1 GiB) is cut into segments of BT x ZPT = 16K symbols, one
// 1024-thread workgroup each (blocks [0, nz) of k_body).  Two phases:
//  A (no waiting): a segment runs zone_one's site deltas and local compaction
//    on its range (neighbour symbols before / after it come from the current
//    zone buffer, where their owners may already have rewritten them in place:
//    token nw reads back as a, since nw exists nowhere else before this merge),
//    and takes an even share of the two mc-long per-merge chores: the stale
//    tail's destroyed pairs ([z - mc, z), read the same way) and the stale-window
//    SOURCE ([n - 2mc - Bp, + mc) of the other buffer) copied into LDS.  It
//    publishes (kept, tail survivors, last kept symbol) as three 8-byte
//    {tag, value} granules (relaxed agent-scope stores: the data is the flag)
//    after every wave drained its loads.
//  B: one wave sweeps all nz segments' granules; then the segment stores its
//    kept symbols at its prefix and the part of the window (the last m source
//    symbols, m = all tail survivors) in its share after the Kz kept ones.  Every
//    read of the other buffer (the window source) happened in phase A, before
//    any segment passes phase B's sweep, so no store overwrites an unread source.
//  Every zone workgroup waits only on zone workgroups, which never wait on body
//  workgroups: with nz <= 64 workgroups they all become resident.
// k_refresh zeroes the granules for the next merge (tag = 1).
template <typename S, bool EXACT, int BT, int NT, int ZPT>
__device__ void zone_seg(DevState* st, DevState* zst, const DevState& gs, const DevState& zs, S* __restrict__ zc,
                         S* __restrict__ zo, ZSegState* zg, uint32_t nz, ZoneLds<S, BT>& L, LdsTab<NT>& lt,
                         const Table& tb, uint32_t a, uint32_t b, uint32_t nw, uint32_t mc,
                         uint64_t* __restrict__ bytes, uint32_t round) {
    (void)round;
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    constexpr uint32_t SEG = (uint32_t)BT * ZPT;
    constexpr int V = ZPT * sizeof(S) / 16;
    static_assert(ZPT <= ZoneDim<S, BT>::ZPT && ZPT * sizeof(S) % 16 == 0, "segment positions per thread");
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    __shared__ uint32_t s_h[3], s_last, s_pre, s_kz, s_m, s_x0;
    const uint32_t seg = blockIdx.x;
    const uint32_t z = zs.n;
    const uint32_t lim = EXACT ? z : z - mc;
    const uint32_t g0 = seg * SEG;
    const uint32_t nh = g0 < z ? (z - g0 < SEG ? z - g0 : SEG) : 0u;   // positions of this segment (0: past the end)
    const uint32_t pid_ab = (a << 16) | b;
    auto unrw = [&](uint32_t v) -> uint32_t { return (v & TM) == nw ? (a | (v & WS)) : v; };
    auto zload = [&](uint32_t p) -> uint32_t { return unrw((uint32_t)((const volatile S*)zc)[p]); };   // old or rewritten
    const uint32_t i0 = (uint32_t)t * ZPT;   // local
    S* xs = reinterpret_cast<S*>(L.xv);
    uint32_t x[ZPT];
    {
        uint4 v[V];
        const uint4* src = reinterpret_cast<const uint4*>(zc + g0 + i0);
        const bool any = i0 < nh;
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = any ? src[k] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int k = 0; k < V; ++k) L.xv[t * V + k] = v[k];
        const S* e = reinterpret_cast<const S*>(v);
#pragma unroll
        for (int k = 0; k < ZPT; ++k) x[k] = i0 + k < nh ? (uint32_t)e[k] : 0u;
    }
    if (t < 3) {   // neighbours g0 - 2, g0 - 1, g0 + nh
        const uint32_t p = t < 2 ? g0 - 2u + (uint32_t)t : g0 + nh;
        const bool ok = nh && (t < 2 ? g0 >= 2u - (uint32_t)t : g0 + nh < z);
        s_h[t] = ok ? zload(p) : 0u;
    }
    // this segment's share of the window source (+ the symbol before it) into LDS
    const uint32_t lw = (mc + nz - 1) / nz, q0 = seg * lw, q1 = q0 + lw < mc ? q0 + lw : mc;   // source [q0, q1)
    const uint64_t src0 = (uint64_t)gs.n + gs.off - gs.poff - 2ull * mc - gs.Bp;
    if (!EXACT && q0 < q1) {
        const uint32_t f = q0 ? q0 - 1u : 0u;   // L.wb[j] = source[f + j]
        for (uint32_t q = f + t; q < q1; q += BT) L.wb[q - f] = zo[src0 + q];
    }
    lds_clear(lt);
    __syncthreads();
    if (t == 0) KT(2);
    auto X = [&](int j) -> uint32_t {   // local position j in [-2, SEG]
        return j < 0 ? s_h[j + 2] : (uint32_t)j < nh ? (uint32_t)xs[j] : ((uint32_t)j == nh ? s_h[2] : 0u);
    };
    if (!EXACT) {   // this segment's share of the stale tail: old pairs destroyed
        const uint32_t lo = lim > 1u ? lim : 1u;
        const uint32_t nt_ = z > lo ? z - lo : 0u, lt_ = (nt_ + nz - 1) / nz;
        const uint32_t p0 = lo + seg * lt_, p1 = p0 + lt_ < z ? p0 + lt_ : z;
        for (uint32_t i = p0 + t; i < p1; i += BT) {
            const uint32_t xi = zload(i);
            if (xi & WS) continue;
            const uint32_t tp = zload(i - 1) & TM, ti = xi & TM;
            if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
        }
    }
    const uint32_t xm2 = X((int)i0 - 2), xm1 = X((int)i0 - 1), nxr = X((int)(i0 + ZPT));
    uint32_t eb = 0, ea = 0;
#pragma unroll
    for (int k = 0; k < ZPT; ++k) {
        eb |= (x[k] == b ? 1u : 0u) << k;
        ea |= ((x[k] & TM) == a ? 1u : 0u) << k;
    }
    const uint32_t gi0 = g0 + i0;
    const uint32_t inb = lane_mask_n(i0, nh, ZPT);
    const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a ? 1u : 0u)) & inb;
    const uint32_t h_m1 = (gi0 >= 1 && i0 <= nh && xm1 == b && (xm2 & TM) == a) ? 1u : 0u;
    const uint32_t h_32 = (nxr == b && (ea >> (ZPT - 1))) ? 1u : 0u;
    const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_32 << (ZPT + 1));
    const uint32_t below = lane_mask_n(gi0, lim, ZPT);
    const uint32_t surv = inb & ~hitm, keep = surv & below;
    const uint32_t rwm = ((hitm >> 1) | (h_32 << (ZPT - 1))) & inb;
    uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
    while (rel) {
        const int k = __ffs(rel) - 1;
        rel &= rel - 1;
        const uint32_t i = i0 + k;
        if (g0 + i == 0) continue;
        const uint32_t xi = X((int)i);
        if (xi & WS) continue;
        const uint32_t xp = X((int)i - 1);
        const bool hm = (hbits >> k) & 1u, h0 = (hbits >> (k + 1)) & 1u, hp = (hbits >> (k + 2)) & 1u;
        const uint32_t tp = xp & TM, ti = xi & TM;
        if (tp && ti && ((tp << 16) | ti) != pid_ab) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
        if (!h0) {
            if (hm) {
                const uint32_t t2 = hp ? nw : ti;
                if (t2) lds_add(lt, tb, st, (nw << 16) | t2, 1u);
            } else if (hp && tp) {
                lds_add(lt, tb, st, (tp << 16) | nw, 1u);
            }
        }
    }
    if (t == 0) KT(3);
    // local exclusive scan of the kept counts; tail survivors; the last kept symbol
    const uint32_t kc = __popc(keep);
    uint32_t incl = kc, tl = __popc(surv & ~below);
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    for (int off = 32; off > 0; off >>= 1) tl += __shfl_xor(tl, off);
    if (lane == 63) L.wsum[wid] = incl;
    if (lane == 0) L.wtail[wid] = tl;
    __syncthreads();
    uint32_t pre = incl - kc, Ks = 0, Ts = 0;
#pragma unroll
    for (int w2 = 0; w2 < BT / 64; ++w2) {
        pre += w2 < wid ? L.wsum[w2] : 0u;
        Ks += L.wsum[w2];
        Ts += L.wtail[w2];
    }
    if (kc && pre + kc == Ks) {   // this thread holds the segment's last kept symbol
        const int hk = 31 - __clz(keep);
        uint32_t xv = x[0];
#pragma unroll
        for (int k = 1; k < ZPT; ++k) xv = k == hk ? x[k] : xv;
        s_last = ((rwm >> hk) & 1u) ? (nw | (xv & WS)) : xv;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's reads of the other buffer are done
    __syncthreads();
    if (t == 0) {
        constexpr unsigned long long TAG = 1ull << 32;
        __hip_atomic_store(&zg->gran[seg][0], TAG | Ks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&zg->gran[seg][1], TAG | Ts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&zg->gran[seg][2], TAG | (Ks ? (s_last | 0x80000000u) : 0u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        KT(7);
    }
    // the new segment assembled in LDS over the old copy (swizzled as in zone_one)
    constexpr uint32_t PV = 16 / sizeof(S), PVL = sizeof(S) == 2 ? 3 : 2;
    auto swz = [](uint32_t o) -> uint32_t {
        const uint32_t c = o >> PVL;
        return ((c ^ ((c >> 3) & 7u)) << PVL) | (o & (PV - 1u));
    };
    uint32_t wsm = 0;
#pragma unroll
    for (int k = 0; k < ZPT; ++k) {
        const bool rw = (rwm >> k) & 1u;
        const uint32_t v = rw ? (nw | (x[k] & WS)) : x[k];
        wsm |= ((x[k] & WS) ? 1u : 0u) << k;
        const uint32_t o = pre + (uint32_t)__popc(keep & ((1u << k) - 1u));
        S* dst = ((keep >> k) & 1u) ? &xs[swz(o)] : &L.trash[lane];
        *dst = (S)v;
    }
    for (uint32_t r = rwm; r; r &= r - 1) {
        const int k = __ffs(r) - 1;
        zc[gi0 + k] = (S)(nw | (((wsm >> k) & 1u) ? WS : 0u));
    }
    // B: every segment's granules (one wave, relaxed sweeps, s_sleep between)
    if (wid == 0) {
        uint32_t gk = 0, gt = 0, gl = 0;
        for (uint32_t it = 0;; ++it) {
            bool ok = true;
            if ((uint32_t)lane < nz) {
                const unsigned long long x0 = __hip_atomic_load(&zg->gran[lane][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long x1 = __hip_atomic_load(&zg->gran[lane][1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long x2 = __hip_atomic_load(&zg->gran[lane][2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = (x0 >> 32) == 1u && (x1 >> 32) == 1u && (x2 >> 32) == 1u;
                gk = (uint32_t)x0;
                gt = (uint32_t)x1;
                gl = (uint32_t)x2;
            }
            if (__all(ok)) break;
            if (it > ZSEG_SPIN) {
                if (lane == 0) atomicOr(&st->err, ERR_SPIN);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const bool in = (uint32_t)lane < nz;
        uint32_t sp = in && (uint32_t)lane < seg ? gk : 0u, sk = in ? gk : 0u, stt = in ? gt : 0u;
        for (int off = 32; off > 0; off >>= 1) {
            sp += __shfl_xor(sp, off);
            sk += __shfl_xor(sk, off);
            stt += __shfl_xor(stt, off);
        }
        const unsigned long long hm = __ballot(in && (gl >> 31));
        if (lane == 0) {
            s_pre = sp;
            s_kz = sk;
            s_m = EXACT ? 0u : stt;
            s_x0 = 0u;
        }
        if (hm && lane == 63 - __clzll(hm)) s_x0 = gl & 0x7FFFFFFFu;   // the last kept survivor overall
    }
    __syncthreads();
    if (t == 0) KT(8);
    const uint32_t P = s_pre, Kz = s_kz, m = s_m;
    for (uint32_t j = t; j < Ks; j += BT) zo[P + j] = xs[swz(j)];
    if (!EXACT && m) {   // the window = source [mc - m, mc) after the Kz kept symbols; this segment's share
        const uint32_t w0 = mc - m, f = q0 ? q0 - 1u : 0u;
        const uint32_t lo = q0 > w0 ? q0 : w0;
        for (uint32_t q = lo + t; q < q1; q += BT) {
            const uint32_t x1 = L.wb[q - f];
            const uint32_t x0 = q == w0 ? s_x0 : (uint32_t)L.wb[q - 1u - f];
            zo[Kz + (q - w0)] = (S)x1;
            if (!(x1 & WS) && (x0 & TM) && (x1 & TM)) lds_add(lt, tb, st, ((x0 & TM) << 16) | (x1 & TM), 1u);
        }
    }
    if (t == 0) KT(9);
    lds_flush(lt, tb, st);
    if (t == 0) {
        KT(4);
        if (seg == 0) {
            zst->m = m;
            zst->valid_total = Kz + m + 1u;
        }
        const uint32_t ws = q1 > q0 ? q1 - q0 : 0u;
        atomicAdd(bytes, (uint64_t)sizeof(S) * ((uint64_t)nh + Ks + 2u * ws + (EXACT ? 0u : mc / nz)));
    }
}

// Selection inside k_body (sector-sparse loop): every workgroup reduces the
// k_refresh partial maxima itself and gets the same merge; the last one commits
// it (log, table slot zeroed, state for k_refresh and the zone kernels).  The
// step counters move on in k_refresh (finish == 2), so nothing a workgroup reads
// here changes under it.  Saves the k_select launch per merge.
// Sharded (cap_list != 0): the zone sits on the last rank only, so the zone checks
// use st->zlast, the zone length every rank learned from the last exchange; a
// merge whose count could overflow the exchange record stalls here, before any
// sector is touched, on every rank alike (the count is global).
struct SelShard {
    uint32_t zf = 5;         // zone rule: z >= max(2 mc + mc_prev, zf mc) + 2 (single GPU: GBPE_ZONE_F, sharded 5)
    uint32_t cap_list = 0;   // 0 = single GPU
    uint32_t zmax = 0;       // the one-workgroup zone limit (sharded zones never run multi-tile)
    uint32_t* nlog = nullptr;
    uint32_t* rec = nullptr; // this rank's exchange record (its list length restarts at 0)
};

template <int BT>
__device__ bool sel_inline(DevState* st, DevState* zst, const uint64_t* __restrict__ part, uint32_t npart,
                           uint32_t round, bool exact, bool zone1, const Table& tb, uint32_t* __restrict__ log,
                           uint32_t* __restrict__ grpsum, uint32_t& a, uint32_t& b, uint32_t& nw, uint32_t& mc,
                           const DevState*& gsnap, const DevState*& zsnap, const SelShard sh = SelShard(),
                           bool commit = true) {
    __shared__ uint64_t s_red[BT / 64];
    constexpr int NW = sizeof(DevState) / 4;
    __shared__ union {
        DevState d;
        uint32_t w[NW];
    } s_g, s_z;
    const int t = threadIdx.x;
    // the partial maxima and snapshots of both states load together (one round
    // trip, not one per field)
    if (t < NW) s_g.w[t] = reinterpret_cast<const uint32_t*>(st)[t];
    else if (zst && t < 2 * NW) s_z.w[t - NW] = reinterpret_cast<const uint32_t*>(zst)[t - NW];
    uint64_t best = 0;
    for (uint32_t i = t; i < npart; i += BT) {
        const uint64_t v = part[i];
        best = v > best ? v : best;
    }
    __syncthreads();
    const DevState& g = s_g.d;
    gsnap = &s_g.d;
    zsnap = &s_z.d;
    if (!(round < g.budget && g.merges_done == round && !g.stop && !g.sp_abort && !g.stall)) return false;
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((t & 63) == 0) s_red[t >> 6] = best;
    __syncthreads();
    best = s_red[0];
#pragma unroll
    for (int w = 1; w < BT / 64; ++w) best = s_red[w] > best ? s_red[w] : best;
    mc = (uint32_t)(best >> 32);
    const uint32_t pid = ~(uint32_t)best;
    a = pid >> 16;
    b = pid & 0xFFFFu;
    nw = g.next_id;
    const bool stop = mc < 2u || nw > 0xFFFFu;                                          // train.wgsl:345-348
    const bool bad = !stop && !exact && g.is_last &&
                     (uint64_t)g.n + g.off - g.poff < 2ull * mc + g.Bp;   // cannot happen
    // zone misfit: this merge's window source must lie in the zone's stale buffer
    // (n - 2mc >= Bp, where n - Bp >= z - mc_prev: the last merge removed <= mc_prev
    // body symbols), and the zone keeps >= zf mc for the merges after it
    const uint32_t mc_prev = sh.cap_list ? g.mc : g.mc_prev;
    const uint64_t zneed = std::max<uint64_t>(2ull * mc + mc_prev, (uint64_t)sh.zf * mc) + 2u;
    const bool abort = !stop && !bad && !exact && ((uint64_t)g.zlast < zneed || (sh.zmax && g.zlast > sh.zmax));
    const uint32_t need = 6u * mc + 64u;   // distinct deltas of one merge <= 4 per site + tail + window
    const bool stall = !stop && !bad && !abort && sh.cap_list && need > sh.cap_list;
    const bool go = !stop && !bad && !abort && !stall;
    // the LAST workgroup commits: block 0 is the zone pass (the launch's longest
    // chain), which then starts without the table probe and the state stores
    if (commit && blockIdx.x == gridDim.x - 1u) {
        if (t == 0) {
            if (stop) {
                st->stop = 1u;
            } else if (bad) {
                atomicOr(&st->err, ERR_SPARSE_WINDOW);
                st->stop = 1u;
            } else if (abort) {
                st->sp_abort = 1u;
            } else if (stall) {   // the host grows the records and redoes this merge
                st->stall = 1u;
                st->need_l = need;
                st->need_w = 0u;
            } else {
                if (sh.nlog) sh.nlog[round] = g.n;
                if (sh.rec) {
                    sh.rec[H_L] = 0u;
                    st->dcount = 0u;
                    st->dused = 0u;
                    st->dfull = 0u;
                }
                const uint32_t idx = table_find(tb, pid);
                if (idx == 0xFFFFFFFFu) {
                    atomicOr(&st->err, ERR_PAIR_MISSING);
                } else {
                    // every (a,b) occurrence is a merge site: count -= mc, atomically, since
                    // other workgroups may already add this merge's stale-window pairs
                    atomicSub(&tb.slots[idx].y, mc);
                    tb.dirty[idx >> BLK_LOG2] = 1u;
                }
                log[round * 4 + 0] = a;
                log[round * 4 + 1] = b;
                log[round * 4 + 2] = nw;
                log[round * 4 + 3] = mc;
                st->a = a;
                st->b = b;
                st->nw = nw;
                st->mc = mc;
                st->new_n = g.n - mc;
                zst->a = a;
                zst->b = b;
                zst->nw = nw;
                zst->mc = mc;
                zst->new_n = exact ? s_z.d.n : s_z.d.n - mc;
                if (!zone1) {   // zone_one (another workgroup of this launch) sets both itself
                    zst->m = 0u;
                    zst->valid_total = 0u;
                }
                zst->merges_done = round + 1u;
                st->sel_round = round + 1u;
            }
        }
        if (go) {   // group sums of a multi-tile zone pass start at zero
            const uint32_t ngrp = (uint32_t)gbpe_div_up(gbpe_div_up(s_z.d.n, TILE), GRP);
            for (uint32_t q = t; q < ngrp; q += BT) grpsum[q * GSTR] = 0u;
        }
    }
    return go;
}

// Body pass: blocks [0, nbody) each own `wpg` consecutive bitmap words of
// (a-row & b-row), tested PW words at a time: the candidate sectors whose pair
// signature may hold (a, b) are merged (one wave per sector).  A fixed grid of
// wide workgroups (about 4 per CU at 1 GiB) instead of one workgroup per 16
// words: the selection each workgroup repeats, and the rounds of workgroup
// scheduling, cost more than the bitmap words themselves (75K words per row at
// 1 GiB).  Blocks >= nbody copy the stale-window source [n - 2mc - Bp, + mc) of
// the zone's other buffer to `wtmp`.
// With `zst` (zone <= ZMAX), block nbody runs the whole zone pass (zone_one) and
// there are no copy blocks: one launch merges body and zone.
constexpr uint32_t SP_PW = 64;               // bitmap words tested per pass (one per lane of wave 0)
constexpr uint32_t SP_CAP = SP_PW * 32;      // candidate sectors per pass
struct BodyCand {
    uint32_t sec[SP_CAP];
    uint2 ext[SP_CAP];
};
template <typename S, int BT>
union BodyLds {   // body workgroups use the candidate arrays, the zone workgroup the zone
    ZoneLds<S, BT> z;
    BodyCand c;
};

// ZSEG: the form for zones of 32K-1M symbols: blocks [0, zone1) run the zone
// segments (zone_seg) beside the body blocks, and zone_one is not compiled in
// (with both, every form spilled to scratch)
template <typename S, bool EXACT, int BT, int ZPT = ZoneDim<S, BT>::ZPT, bool ZSEG = false>
__global__ __launch_bounds__(BT) void k_body(DevState* st, uint32_t round, S* __restrict__ body, uint2* __restrict__ sec,
                                              uint32_t* __restrict__ bits, uint32_t W, uint32_t wpg,
                                              uint32_t* __restrict__ sig, Table tb, uint32_t nbody,
                                              const S* __restrict__ zoth, S* __restrict__ wtmp,
                                              uint32_t clog, DevState* zst, S* __restrict__ zcur, uint32_t zone1,
                                              const uint64_t* __restrict__ part, uint32_t npart, uint32_t* __restrict__ log,
                                              uint32_t* __restrict__ grpsum, uint64_t* __restrict__ wg_bytes,
                                              Table dtb, SelShard sh, uint32_t* __restrict__ lmul,
                                              ZSegState* __restrict__ zg = nullptr) {
    constexpr int KB_LT = ZSEG ? 4096 : LTAB_T;
    __shared__ LdsTab<KB_LT> lt;
    __shared__ BodyLds<S, BT> u;
    __shared__ uint32_t s_ntok, s_n, s_any, s_rm[BT / 64];
    __shared__ uint64_t s_mv[BT / 64];
    constexpr int QPT = SP_CAP / BT;   // candidates per thread in the signature test
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    uint32_t a, b, nw, mc;
    if (t == 0) KT(0);
    const DevState *gs, *zs;   // this workgroup's snapshots of the states at launch (LDS)
    if (!sel_inline<BT>(st, zst, part, npart, round, EXACT, zone1 != 0, tb, log, grpsum, a, b, nw, mc, gs, zs, sh))
        return;
    if (t == 0) KT(1);
    // the zone workgroup is dispatched first (block 0 when zone1): it is the longest
    // single chain of the merge, and later blocks of a large grid start later
    const uint32_t bid = blockIdx.x - zone1;
    // deltas go to the replica (single GPU) or to the per-merge delta table (sharded)
    if constexpr (ZSEG) {
        if (blockIdx.x < zone1) {
            zone_seg<S, EXACT, BT, KB_LT, 16>(st, zst, *gs, *zs, zcur, (S*)zoth, zg, zone1, u.z, lt, dtb, a, b, nw, mc,
                                             wg_bytes + nbody, round);
            if (t == 0) {
                KT(5);
                KTV(6, 2);
            }
            return;
        }
    } else {
        if (zone1 == 1 && blockIdx.x == 0) {
            zone_one<S, EXACT, BT, KB_LT, ZPT>(st, zst, *gs, *zs, zcur, (S*)zoth, u.z, lt, dtb, a, b, nw, mc,
                                                 wg_bytes + nbody, round);
            if (t == 0) {
                KT(5);
                KTV(6, 2);
            }
            return;
        }
    }
    if (bid >= nbody) {
        const uint64_t src0 = (uint64_t)gs->n + gs->off - gs->poff - 2ull * mc - gs->Bp;
        const uint64_t stride = (uint64_t)(gridDim.x - nbody) * BT;
        for (uint64_t v = (uint64_t)(bid - nbody) * BT + t; v < mc; v += stride) wtmp[v] = zoth[src0 + v];
        if (t == 0) {
            KT(5);
            KTV(6, 3);
        }
        return;
    }
    const uint32_t pid_ab = (a << 16) | b;
    BodyCand& cb = u.c;
    lds_clear(lt);
    if (t == 0) s_any = 0u;
    uint32_t removed = 0, ncand_all = 0;
    uint64_t moved = 0, rd = 0;   // sector symbols read + rewritten (wave-uniform); extents + signature words read
    const uint32_t w_beg = bid * wpg, w_end = w_beg + wpg < W ? w_beg + wpg : W;
    for (uint32_t w0 = w_beg; w0 < w_end; w0 += SP_PW) {
        __syncthreads();   // the previous pass is done with s_ntok / s_n / the candidate arrays
        if (t == 0) {
            s_ntok = 0u;
            s_n = 0u;
        }
        __syncthreads();
        if (t < (int)SP_PW && w0 + t < w_end) {   // token candidates
            const uint32_t w = w0 + t;
            uint32_t c = bits[(uint64_t)a * W + w] & bits[(uint64_t)b * W + w];
            if (c) {
                uint32_t pos = atomicAdd(&s_ntok, (uint32_t)__popc(c));
                while (c) {
                    const int bit = __ffs(c) - 1;
                    c &= c - 1;
                    cb.sec[pos++] = w * 32u + (uint32_t)bit;
                }
            }
        }
        __syncthreads();
        const uint32_t ntok = s_ntok;
        if (t == 0) KT(2);
        if (ntok == 0) continue;   // block-uniform
        rd += 16ull * ntok;
        // signature filter: this thread's candidates (their extents load alongside)
        // into registers, then compacted in place
        uint32_t cs[QPT];
        uint2 ce[QPT];
        bool ck[QPT];
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            const uint32_t j = (uint32_t)t + (uint32_t)q * BT;
            cs[q] = j < ntok ? cb.sec[j] : SP_INV;
        }
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            ck[q] = false;
            if (cs[q] != SP_INV) {
                ce[q] = sec[cs[q]];
                ck[q] = sig_has(sig + (uint64_t)cs[q] * SP_SIGW, pid_ab);
            }
        }
        __syncthreads();   // every candidate is read before the list is rewritten
#pragma unroll
        for (int q = 0; q < QPT; ++q)
            if (ck[q]) {
                const uint32_t qq = atomicAdd(&s_n, 1u);
                cb.sec[qq] = cs[q];
                cb.ext[qq] = ce[q];
            }
        __syncthreads();
        const uint32_t ncand = s_n;
        if (t == 0) KT(3);
        if (ncand == 0) continue;   // block-uniform
        ncand_all += ncand;
        if (t == 0) s_any = 1u;
        // software-pipelined: a wave's next sector loads while it merges this one
        uint32_t nf[5], nfm[4];
        if ((uint32_t)wid < ncand)
            sector_first<S>(body + cb.ext[wid].x, lmul ? lmul + cb.ext[wid].x : nullptr, cb.ext[wid].y, nf, nfm);
        for (uint32_t j = wid; j < ncand; j += BT / 64) {
            const uint32_t sct = cb.sec[j];
            const uint2 e = cb.ext[j];
            uint32_t cf[5], cfm[4];
#pragma unroll
            for (int k = 0; k < 5; ++k) cf[k] = nf[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) cfm[k] = nfm[k];
            if (j + BT / 64 < ncand) {
                const uint2 en = cb.ext[j + BT / 64];
                sector_first<S>(body + en.x, lmul ? lmul + en.x : nullptr, en.y, nf, nfm);
            }
            uint32_t out = 0;
            const uint32_t r = body_sector<S, KB_LT>(body + e.x, lmul ? lmul + e.x : nullptr, e.y, a, b, nw, lt, dtb, st,
                                              sig + (uint64_t)sct * SP_SIGW, out, cf, cfm);
            moved += (uint64_t)(sizeof(S) + (lmul ? 4u : 0u)) * (e.y + (r ? out : 0u));
            if (r) {
                removed += r;
                if (lane == 0) {
                    if (clog) atomicAdd(&st->hitsec, 1u);
                    sec[sct].y = out;
                    atomicOr(&bits[(uint64_t)nw * W + (sct >> 5)], 1u << (sct & 31u));
                }
            }
        }
    }
    __syncthreads();
    if (t == 0) KT(4);
    if (!s_any) {   // block-uniform: no candidate survived the filters
        if (t == 0) {
            if (rd) atomicAdd(&wg_bytes[bid], rd);
            KT(5);
            KTV(6, 0);
        }
        return;
    }
    if (t == 0 && clog) atomicAdd(&st->cand, ncand_all);
    lds_flush(lt, dtb, st);
    if (lane == 0) {
        s_rm[wid] = removed;
        s_mv[wid] = moved;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t r = 0;
        uint64_t mv = rd;
        for (int w2 = 0; w2 < BT / 64; ++w2) {
            r += s_rm[w2];
            mv += s_mv[w2];
        }
        if (r) atomicAdd(&st->body_rm, r);
        atomicAdd(&wg_bytes[bid], mv);   // this workgroup's own counter
        KT(5);
        KTV(6, 1 | (ncand_all << 8));
    }
}

// ── persistent tail loop ──
// Late merges (a few hundred sites in a handful of distinct words, a zone of a
// few K symbols) cost launches and dependent round trips, not bytes: k_body +
// k_refresh spend ~20 us per merge at 1 GiB on ~10 candidate sectors.  k_tail is
// ONE 1024-thread workgroup that runs a whole step's merges back to back.  It is
// the only writer of the pair table while it runs, so
//   * selection reduces group maxima kept in LDS (64 argmax blocks per group)
//     instead of a k_refresh pass and its partial maxima;
//   * count deltas reach the table as plain read-modify-writes; each raises its
//     block maximum (atomicMax) or, when it lowers the block's holder, has the
//     block re-maxed from its 2048 slots by one wave;
//   * the body pass (every bitmap word of rows a and b in one load, signatures,
//     one wave per candidate sector) and the zone pass (zone_one) share one LDS
//     delta table and one flush.
// It leaves the step early — the host finishes it with k_body — when a merge's
// candidate sectors or re-maxed blocks outgrow its LDS lists.
#ifdef GBPE_TAIL_LOOP
constexpr int TL_BT = 1024;
constexpr int TL_LT = 4096;               // LDS delta table (body + zone deltas of one merge)
constexpr uint32_t TL_GRP = 6;            // log2 argmax blocks per group
constexpr uint32_t TL_MAXG = 256;         // groups: tables of up to 2^25 slots
constexpr uint32_t TL_RS = 1024;          // re-maxed blocks per merge
constexpr uint32_t TL_CAND = 8192;        // candidate sectors per merge (token bitmap)
constexpr uint32_t TL_FILT = 3072;        // ... passing the signature filter
enum : uint32_t { TL_EXIT_NONE = 0, TL_EXIT_CAND = 1, TL_EXIT_REMAX = 2, TL_EXIT_LDS = 3 };

struct TailBody {   // the body pass's lists (the zone pass reuses this LDS)
    uint32_t cand[TL_CAND];
    uint32_t fsec[TL_FILT];
    uint2 fext[TL_FILT];
};
template <typename S>
union TailU {
    ZoneLds<S, TL_BT> z;
    TailBody c;
};
static_assert(sizeof(TailBody) <= sizeof(ZoneLds<uint32_t, TL_BT>), "the body lists share the zone's LDS");

__device__ __forceinline__ uint64_t tl_key(uint32_t cnt, uint32_t pid) {
    return (int32_t)cnt > 0 ? (((uint64_t)cnt << 32) | (uint32_t)~pid) : 0ull;
}

template <typename S, bool EXACT, int ZPT>
__global__ __launch_bounds__(TL_BT) void k_tail(DevState* st, DevState* zst, S* __restrict__ body, uint32_t* __restrict__ lmul,
                                                uint2* __restrict__ sec, uint32_t* __restrict__ bits, uint32_t W,
                                                uint32_t wused, uint32_t* __restrict__ sig, Table tb, S* __restrict__ zb0,
                                                S* __restrict__ zb1, uint32_t* __restrict__ log,
                                                uint64_t* __restrict__ bytes, uint32_t* __restrict__ tstat) {
    __shared__ TailU<S> u;
    __shared__ LdsTab<TL_LT> lt;
    __shared__ uint64_t gmax[TL_MAXG];
    __shared__ uint32_t rs[TL_RS], rsmark[(TL_MAXG << TL_GRP) / 32], gmark[TL_MAXG / 32];
    __shared__ uint32_t s_nrs, s_ntok, s_nf, s_rm, s_exit, s_used, s_idx, zout[2];
    __shared__ uint64_t s_red[TL_BT / 64];
    constexpr int NW = sizeof(DevState) / 4;
    constexpr uint32_t NWAVE = TL_BT / 64;
    __shared__ union {
        DevState d;
        uint32_t w[NW];
    } s_g, s_z;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t ngrp = (tb.nblk + (1u << TL_GRP) - 1) >> TL_GRP;
    if (t < NW) s_g.w[t] = reinterpret_cast<const uint32_t*>(st)[t];
    else if (t < 2 * NW) s_z.w[t - NW] = reinterpret_cast<const uint32_t*>(zst)[t - NW];
    for (uint32_t g = wid; g < ngrp; g += NWAVE) {   // group maxima from the (exact) block maxima
        const uint32_t blk = (g << TL_GRP) + (uint32_t)lane;
        uint64_t v = blk < tb.nblk ? tb.bmax[blk] : 0ull;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(v, off);
            v = o > v ? o : v;
        }
        if (lane == 0) gmax[g] = v;
    }
    for (uint32_t i = t; i < (TL_MAXG << TL_GRP) / 32; i += TL_BT) rsmark[i] = 0u;
    if (t < (int)(TL_MAXG / 32)) gmark[t] = 0u;
    if (t == 0) {
        s_exit = TL_EXIT_NONE;
        s_used = 0u;
    }
    __syncthreads();
    DevState& g = s_g.d;
    DevState& z = s_z.d;
    const uint32_t K = g.budget;
    uint64_t mybytes = 0;
    auto remax_mark = [&](uint32_t blk) {   // queue a block for re-maxing (once per merge)
        const uint32_t bit = 1u << (blk & 31u);
        if (!(atomicOr(&rsmark[blk >> 5], bit) & bit)) {
            const uint32_t q = atomicAdd(&s_nrs, 1u);
            if (q < TL_RS) rs[q] = blk;
            else tb.dirty[blk] = 1u;   // k_refresh after the kernel re-maxes it; the loop stops after this merge
        }
    };
    uint32_t r = g.merges_done;
    for (; r < K; ++r) {
        if (g.stop || g.sp_abort || g.err) break;   // (uniform: LDS state, read after a barrier)
        if (t == 0) TKT(0);
        // ── selection: group maxima (LDS) ──
        uint64_t best = 0;
        for (uint32_t i = t; i < ngrp; i += TL_BT) best = gmax[i] > best ? gmax[i] : best;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(best, off);
            best = o > best ? o : best;
        }
        if (lane == 0) s_red[wid] = best;
        if (t == 0) {
            s_ntok = 0u;
            s_nf = 0u;
            s_rm = 0u;
            s_nrs = 0u;
        }
        lds_clear(lt);
        __syncthreads();
        best = s_red[0];
#pragma unroll
        for (uint32_t w2 = 1; w2 < NWAVE; ++w2) best = s_red[w2] > best ? s_red[w2] : best;
        const uint32_t mc = (uint32_t)(best >> 32), pid = ~(uint32_t)best, a = pid >> 16, b = pid & 0xFFFFu;
        const uint32_t nw = g.next_id;
        if (mc < 2u || nw > 0xFFFFu) {   // train.wgsl:345-348
            if (t == 0) g.stop = 1u;
            break;
        }
        if (t == 0) TKT(1);
        if (!EXACT) {
            if ((uint64_t)g.n < 2ull * mc + g.Bp) {   // cannot happen (k_body's invariant)
                if (t == 0) {
                    g.err |= ERR_SPARSE_WINDOW;
                    g.stop = 1u;
                }
                break;
            }
            if ((uint64_t)z.n < 5ull * mc + 2u) {   // zone misfit: the host goes dense
                if (t == 0) g.sp_abort = 1u;
                break;
            }
        }
        // ── body candidates: every bitmap word of rows a and b at once (thread 0 finds (a,b)'s slot first) ──
        if (t == 0) s_idx = table_find(tb, pid);
        for (uint32_t w = t; w < wused; w += TL_BT) {
            uint32_t c = bits[(uint64_t)a * W + w] & bits[(uint64_t)b * W + w];
            if (c) {
                uint32_t pos = atomicAdd(&s_ntok, (uint32_t)__popc(c));
                for (; c; c &= c - 1, ++pos)
                    if (pos < TL_CAND) u.c.cand[pos] = w * 32u + (uint32_t)(__ffs(c) - 1);
            }
        }
        __syncthreads();
        const uint32_t ntok = s_ntok;
        if (t == 0) {
            TKT(2);
            TKTV(10, ntok);
        }
        if (ntok > TL_CAND) {   // nothing of merge r is committed yet
            if (t == 0) s_exit = TL_EXIT_CAND;
            break;
        }
        for (uint32_t j = t; j < ntok; j += TL_BT) {   // signature filter (+ extents)
            const uint32_t k = u.c.cand[j];
            const uint2 e = sec[k];
            if (sig_has(sig + (uint64_t)k * SP_SIGW, pid)) {
                const uint32_t q = atomicAdd(&s_nf, 1u);
                if (q < TL_FILT) {
                    u.c.fsec[q] = k;
                    u.c.fext[q] = e;
                }
            }
        }
        if (t == 0) mybytes += 16ull * ntok;
        __syncthreads();
        const uint32_t nf = s_nf;
        if (t == 0) {
            TKT(3);
            TKTV(11, nf);
        }
        if (nf > TL_FILT) {
            if (t == 0) s_exit = TL_EXIT_CAND;
            break;
        }
        // ── commit: the log (thread 0); count(a,b) -= mc and the re-max of its block and
        //    group by the last wave, while the others merge sectors ──
        const uint32_t idx = s_idx;
        if (t == 0) {
            if (idx == 0xFFFFFFFFu) g.err |= ERR_PAIR_MISSING;
            log[r * 4 + 0] = a;
            log[r * 4 + 1] = b;
            log[r * 4 + 2] = nw;
            log[r * 4 + 3] = mc;
        }
        if (wid == (int)NWAVE - 1 && idx != 0xFFFFFFFFu) {
            constexpr int NV = (1 << BLK_LOG2) / 2 / 64;   // 16-byte loads per lane
            const uint32_t blk = idx >> BLK_LOG2, gq = blk >> TL_GRP, gb = (gq << TL_GRP) + (uint32_t)lane;
            const uint32_t cnt_new = tb.slots[idx].y - mc;
            const uint4* sl = reinterpret_cast<const uint4*>(tb.slots + ((uint64_t)blk << BLK_LOG2));
            uint4 e[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) e[k] = sl[lane + k * 64];
            const uint64_t gbm = gb < tb.nblk && gb != blk ? tb.bmax[gb] : 0ull;
            if (lane == 0) tb.slots[idx].y = cnt_new;
            uint64_t bst = 0;
            uint32_t live = 0;
#pragma unroll
            for (int k = 0; k < NV; ++k) {   // (a,b)'s slot with its new count
                const uint32_t s0 = ((uint32_t)(lane + k * 64) << 1) + ((blk << BLK_LOG2));
                const uint32_t c1 = s0 == idx ? cnt_new : e[k].y, c2 = s0 + 1 == idx ? cnt_new : e[k].w;
                const uint64_t k1 = e[k].x ? tl_key(c1, e[k].x) : 0ull, k2 = e[k].z ? tl_key(c2, e[k].z) : 0ull;
                bst = k1 > bst ? k1 : bst;
                bst = k2 > bst ? k2 : bst;
                live += (k1 ? 1u : 0u) + (k2 ? 1u : 0u);
            }
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t o = __shfl_xor(bst, off);
                bst = o > bst ? o : bst;
                live += __shfl_xor(live, off);
            }
            uint64_t gv = gbm > bst ? gbm : bst;
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t o = __shfl_xor(gv, off);
                gv = o > gv ? o : gv;
            }
            if (lane == 0) {
                tb.bmax[blk] = bst;
                tb.blive[blk] = live;
                gmax[gq] = gv;
            }
        }
        // ── body sectors: one wave each, the next one's loads in flight ──
        {
            uint32_t removed = 0;
            uint64_t moved = 0;
            uint32_t nf5[5], nfm[4];
            if ((uint32_t)wid < nf)
                sector_first<S>(body + u.c.fext[wid].x, lmul ? lmul + u.c.fext[wid].x : nullptr, u.c.fext[wid].y, nf5, nfm);
            for (uint32_t j = wid; j < nf; j += NWAVE) {
                const uint32_t sct = u.c.fsec[j];
                const uint2 e = u.c.fext[j];
                uint32_t cf[5], cfm[4];
#pragma unroll
                for (int k = 0; k < 5; ++k) cf[k] = nf5[k];
#pragma unroll
                for (int k = 0; k < 4; ++k) cfm[k] = nfm[k];
                if (j + NWAVE < nf) {
                    const uint2 en = u.c.fext[j + NWAVE];
                    sector_first<S>(body + en.x, lmul ? lmul + en.x : nullptr, en.y, nf5, nfm);
                }
                uint32_t out = 0;
                const uint32_t rr = body_sector<S, TL_LT>(body + e.x, lmul ? lmul + e.x : nullptr, e.y, a, b, nw, lt, tb, st,
                                                         sig + (uint64_t)sct * SP_SIGW, out, cf, cfm);
                moved += (uint64_t)(sizeof(S) + (lmul ? 4u : 0u)) * (e.y + (rr ? out : 0u));
                if (rr) {
                    removed += rr;
                    if (lane == 0) {
                        sec[sct].y = out;
                        atomicOr(&bits[(uint64_t)nw * W + (sct >> 5)], 1u << (sct & 31u));
                    }
                }
            }
            if (lane == 0) {
                if (removed) atomicAdd(&s_rm, removed);
                mybytes += moved;
            }
        }
        __syncthreads();
        if (t == 0) TKT(4);
        // ── zone (the same delta table) ──
        S* zc = (r & 1u) ? zb1 : zb0;
        S* zo = (r & 1u) ? zb0 : zb1;
        zone_one<S, EXACT, TL_BT, TL_LT, ZPT>(st, zst, g, z, zc, zo, u.z, lt, tb, a, b, nw, mc, bytes, r, zout);
        __syncthreads();
        if (t == 0) TKT(5);
        // ── flush: plain read-modify-writes (the only writer), block maxima kept exact ──
        {
            uint32_t kk[TL_LT / TL_BT], vv[TL_LT / TL_BT];
#pragma unroll
            for (int j = 0; j < TL_LT / TL_BT; ++j) {
                kk[j] = lt.key[t + j * TL_BT];
                vv[j] = lt.val[t + j * TL_BT];
            }
#pragma unroll
            for (int j = 0; j < TL_LT / TL_BT; ++j) {
                const uint32_t p = kk[j], d = vv[j];
                if (!p || !d) continue;
                const uint32_t h = gbpe_fmix32(p) & tb.mask;
                uint32_t idx = 0xFFFFFFFFu, old = 0;
                for (uint32_t q = 0; q <= tb.mask; ++q) {
                    const uint32_t i2 = (h + ((q * (q + 1)) >> 1)) & tb.mask;
                    uint32_t k2 = tb.slots[i2].x;
                    if (k2 == 0u) {
                        k2 = atomicCAS(&tb.slots[i2].x, 0u, p);   // another new pair may race for the slot
                        if (k2 == 0u) {
                            atomicAdd(&s_used, 1u);
                            idx = i2;
                            old = 0u;
                            break;
                        }
                    }
                    if (k2 == p) {
                        idx = i2;
                        old = tb.slots[i2].y;
                        break;
                    }
                }
                if (idx == 0xFFFFFFFFu) {
                    atomicOr(&g.err, ERR_TABLE_FULL);
                    continue;
                }
                const uint32_t nv = old + d;
                tb.slots[idx].y = nv;
                const uint32_t blk = idx >> BLK_LOG2;
                const uint64_t bm = __hip_atomic_load(&tb.bmax[blk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t ok = tl_key(old, p), nk = tl_key(nv, p);
                if (nk > bm) {
                    atomicMax(&tb.bmax[blk], nk);
                    atomicMax(&gmax[blk >> TL_GRP], nk);
                } else if (nk < ok && ok == bm) {
                    remax_mark(blk);
                }
            }
        }
        __syncthreads();
        if (t == 0) {
            TKT(6);
            TKTV(9, s_nrs);
        }
        // ── re-max queued blocks (one wave each), then their groups ──
        if (s_nrs) {
            const uint32_t nrs = s_nrs < TL_RS ? s_nrs : TL_RS;
            constexpr int NV = (1 << BLK_LOG2) / 2 / 64;   // 16-byte loads per lane
            for (uint32_t q = wid; q < nrs; q += NWAVE) {
                const uint32_t blk = rs[q];
                const uint4* sl = reinterpret_cast<const uint4*>(tb.slots + ((uint64_t)blk << BLK_LOG2));
                uint4 e[NV];
#pragma unroll
                for (int k = 0; k < NV; ++k) e[k] = sl[lane + k * 64];
                uint64_t bst = 0;
                uint32_t live = 0;
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const uint64_t k1 = e[k].x ? tl_key(e[k].y, e[k].x) : 0ull, k2 = e[k].z ? tl_key(e[k].w, e[k].z) : 0ull;
                    bst = k1 > bst ? k1 : bst;
                    bst = k2 > bst ? k2 : bst;
                    live += (k1 ? 1u : 0u) + (k2 ? 1u : 0u);
                }
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(bst, off);
                    bst = o > bst ? o : bst;
                    live += __shfl_xor(live, off);
                }
                if (lane == 0) {
                    tb.bmax[blk] = bst;
                    tb.blive[blk] = live;
                    atomicOr(&gmark[blk >> (TL_GRP + 5)], 1u << ((blk >> TL_GRP) & 31u));
                }
            }
            __syncthreads();
            for (uint32_t gq = wid; gq < ngrp; gq += NWAVE) {
                if (!((gmark[gq >> 5] >> (gq & 31u)) & 1u)) continue;   // wave-uniform
                const uint32_t blk = (gq << TL_GRP) + (uint32_t)lane;
                uint64_t v = blk < tb.nblk ? __hip_atomic_load(&tb.bmax[blk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(v, off);
                    v = o > v ? o : v;
                }
                if (lane == 0) gmax[gq] = v;
            }
            __syncthreads();
            if (t == 0) TKT(7);
            for (uint32_t i = t; i < (TL_MAXG << TL_GRP) / 32; i += TL_BT) rsmark[i] = 0u;
            if (t < (int)(TL_MAXG / 32)) gmark[t] = 0u;
        }
        // ── state (thread 0): the k_refresh (finish 2) bookkeeping ──
        if (t == 0) {
            const uint32_t m = zout[0], zkeep = zout[1];
            const uint32_t n = g.n - mc, B = g.B - s_rm;
            g.tail_total += m;
            g.Bp = g.B;
            g.B = B;
            g.n = n;
            g.new_n = n;
            g.a = a;
            g.b = b;
            g.nw = nw;
            g.mc = mc;
            z.n = n - B;
            g.zlast = z.n;
            if (z.n != zkeep) {
                g.err |= ERR_COUNT_MISMATCH;
                g.stop = 1u;
            }
            g.next_id = nw + 1u;
            g.epoch += 1u;
            g.merges_done = r + 1u;
            z.merges_done = r + 1u;
            if (s_nrs > TL_RS) s_exit = TL_EXIT_REMAX;
            if (lt.ovf) s_exit = TL_EXIT_LDS;
        }
        __syncthreads();
        if (s_exit != TL_EXIT_NONE) {   // dirty blocks left for the host's k_refresh
            ++r;
            break;
        }
    }
    __syncthreads();
    if (t == 0) {
        g.body_rm = 0u;
        tstat[0] = g.merges_done;
        tstat[1] = s_exit;
    }
    if (mybytes) atomicAdd(bytes, mybytes);
    __syncthreads();
    // the states back (`used` by an add: an overflowing LDS table inserted through table_add)
    constexpr int WUSED = (int)(offsetof(DevState, used) / 4);
    if (t < NW) {
        if (t != WUSED) reinterpret_cast<uint32_t*>(st)[t] = s_g.w[t];
    } else if (t < 2 * NW) {
        reinterpret_cast<uint32_t*>(zst)[t - NW] = s_z.w[t - NW];
    }
    if (t == 0 && s_used) atomicAdd(&st->used, s_used);
}
#endif  // GBPE_TAIL_LOOP

// dense → sparse: the last position at or before `lim` that no counted pair can
// span — a word start, or a token-0 symbol on either side (one workgroup,
// backwards).  The 0s count: the stale window of a huge merge is a 0 run of up
// to ~mc symbols (C5's first merge: ~180M), which a word-start-only search
// crossed at 1024 symbols per round (25 ms per entry / shrink).
template <typename S>
__global__ __launch_bounds__(1024) void k_sp_zone_start(const S* __restrict__ cur, uint32_t lim, uint32_t* __restrict__ out) {
    __shared__ uint32_t s_found;
    if (threadIdx.x == 0) s_found = 0u;
    __syncthreads();
    for (int64_t hi = lim; hi >= 1; hi -= 1024) {
        const int64_t i = hi - (int64_t)threadIdx.x;
        const uint32_t x = i >= 1 ? (uint32_t)cur[i] : 0u, p = i >= 1 ? (uint32_t)cur[i - 1] : 0u;
        if (i >= 1 && ((x & Sym<S>::WS) || !(x & Sym<S>::TM) || !(p & Sym<S>::TM))) atomicMax(&s_found, (uint32_t)i);
        __syncthreads();
        const uint32_t f = s_found;
        __syncthreads();
        if (f) break;
    }
    if (threadIdx.x == 0) *out = s_found;   // 0 = none
}

// window j of a body region [base, base + len) covers [base + j*SEC, +SEC); its
// sector starts at the window's first word start or 0 symbol (window 0: at
// `base`, which is a word start or the stream's first symbol).  No counted pair
// spans either: pairs never cross a word start, and none holds token 0 — the
// stale windows the reference compaction leaves are long 0 runs
// that would otherwise make one sector of up to ~10^6 symbols.  One wave per
// window.
template <typename S>
__global__ __launch_bounds__(TPB) void k_sp_sectors(const S* __restrict__ body, uint32_t base, uint32_t len, uint32_t SEC,
                                                    uint32_t* __restrict__ starts, uint32_t nwin) {
    const uint32_t j = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (j >= nwin) return;
    const uint64_t end = (uint64_t)base + len;
    const uint64_t lo = (uint64_t)base + (uint64_t)j * SEC, hi = lo + SEC < end ? lo + SEC : end;
    uint32_t found = j == 0 ? base : SP_INV;
    for (uint64_t b0 = lo; b0 < hi && found == SP_INV; b0 += 64) {
        const uint64_t i = b0 + lane;
        uint32_t x = i < hi ? (uint32_t)body[i] : 1u;
        const bool ws = (x & Sym<S>::WS) || x == 0u;
        const unsigned long long m = __ballot(ws);
        if (m) found = (uint32_t)(b0 + (uint64_t)(__ffsll((long long)m) - 1));
    }
    if (lane == 0) starts[j] = found;
}

__global__ void k_sp_sector_len(const uint32_t* __restrict__ starts, uint32_t nwin, uint32_t end, uint2* __restrict__ sec) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nwin) return;
    const uint32_t st = starts[k];
    if (st == SP_INV) {
        sec[k] = make_uint2(0u, 0u);
        return;
    }
    uint32_t e = end;
    for (uint32_t j = k + 1; j < nwin; ++j)   // windows inside one long word have no start
        if (starts[j] != SP_INV) {
            e = starts[j];
            break;
        }
    sec[k] = make_uint2(st, e - st);
}

// presence bits of every token (with `bits`) and the pair signature of sectors
// [k0, k0 + nk), one wave per sector.  The signature is built in LDS and stored
// whole (one 128-B line per sector); bitmap words are tested before the atomic.
template <typename S>
__global__ __launch_bounds__(TPB) void k_sp_bits(const S* __restrict__ body, const uint2* __restrict__ sec, uint32_t k0,
                                                 uint32_t nk, uint32_t* __restrict__ bits, uint32_t W,
                                                 uint32_t* __restrict__ sig) {
    __shared__ uint32_t ssig[TPB / 64][SP_SIGW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t k = k0 + blockIdx.x * (TPB / 64) + wid;
    const bool live = k < k0 + nk;
    if (lane < (int)SP_SIGW) ssig[wid][lane] = 0u;
    __syncthreads();
    if (live) {
        const uint2 e = sec[k];
        const uint32_t bit = 1u << (k & 31u);
        uint32_t* col = bits ? bits + (k >> 5) : nullptr;
        for (uint32_t j = lane; j < e.y; j += 64) {
            const uint32_t x = body[e.x + j];
            const uint32_t tok = x & Sym<S>::TM;
            if (col) {
                uint32_t* wp = col + (uint64_t)tok * W;
                if (!(*wp & bit)) atomicOr(wp, bit);
            }
            if (j && !(x & Sym<S>::WS)) {
                const uint32_t tp = body[e.x + j - 1] & Sym<S>::TM;
                if (tp && tok) sig_set(ssig[wid], (tp << 16) | tok);
            }
        }
    }
    __syncthreads();
    if (live && lane < (int)SP_SIGW) sig[(uint64_t)k * SP_SIGW + lane] = ssig[wid][lane];
}

// token bitmap of whole columns (a full rebuild over a zeroed bitmap): one
// workgroup per 32-sector column gathers token -> sector mask in LDS, then
// writes each present token's word once (plain stores; the column is its own).
// Tokens beyond the LDS table's reach take a global atomicOr instead.
constexpr int COLT = 8192;
template <typename S>
__global__ __launch_bounds__(TPB) void k_sp_colbits(const S* __restrict__ body, const uint2* __restrict__ sec, uint32_t nsec,
                                                    uint32_t* __restrict__ bits, uint32_t W) {
    __shared__ uint32_t key[COLT], msk[COLT];
    for (int i = threadIdx.x; i < COLT; i += TPB) {
        key[i] = 0xFFFFFFFFu;
        msk[i] = 0u;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t c = blockIdx.x;
    for (uint32_t q = wid; q < 32; q += TPB / 64) {
        const uint32_t k = c * 32 + q;
        if (k >= nsec) break;
        const uint2 e = sec[k];
        for (uint32_t j = lane; j < e.y; j += 64) {
            const uint32_t tok = body[e.x + j] & Sym<S>::TM;
            uint32_t h = gbpe_fmix32(tok) & (COLT - 1);
            bool done = false;
            for (int p = 0; p < 32 && !done; ++p) {
                const uint32_t o = atomicCAS(&key[h], 0xFFFFFFFFu, tok);
                if (o == 0xFFFFFFFFu || o == tok) {
                    atomicOr(&msk[h], 1u << q);
                    done = true;
                }
                h = (h + 1) & (COLT - 1);
            }
            if (!done) atomicOr(&bits[(uint64_t)tok * W + c], 1u << q);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < COLT; i += TPB)
        if (key[i] != 0xFFFFFFFFu) atomicOr(&bits[(uint64_t)key[i] * W + c], msk[i]);
}

// sparse → dense: sector counts, then a gather at the scanned offsets (one wave per sector)
__global__ void k_sp_counts(const uint2* __restrict__ sec, uint32_t nsec, uint32_t* __restrict__ cnt) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nsec) cnt[k] = sec[k].y;
}

template <typename S>
__global__ __launch_bounds__(TPB) void k_sp_gather(const S* __restrict__ body, const uint2* __restrict__ sec, uint32_t nsec,
                                                   const uint32_t* __restrict__ loc, const uint64_t* __restrict__ blk,
                                                   S* __restrict__ dst) {
    const uint32_t k = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nsec) return;
    const uint2 e = sec[k];
    const uint64_t off = (uint64_t)loc[k] + blk[k / SCAN_BLK];
    for (uint32_t j = lane; j < e.y; j += 64) dst[off + j] = body[e.x + j];
}

#include "lexicon.h"

}  // namespace

// ─── host side ──────────────────────────────────────────────────────────────


struct gbpe_trainer {
    gbpe_ctx* ctx = nullptr;
    bool u16 = true;
    uint32_t bps = 2;            // bytes per symbol
    uint64_t n0 = 0, cap_syms = 0;
    uint64_t n_prev0 = 0;        // created from a state: its previous-stream length (export before any merge)
    void* buf[2] = {nullptr, nullptr};
    int cur = 0;                 // index of the buffer holding the stream
    uint32_t n = 0;              // host copy of the stream length
    uint32_t needed = 0, done = 0;
    bool stop = false;
    uint32_t flags = 0, batch = GBPE_BATCH_SIZE;
    DevState* st = nullptr;
    DevState* h_st = nullptr;    // pinned
    uint32_t* d_log = nullptr;
    uint32_t* h_log = nullptr;   // pinned
    Table tb{};
    uint32_t table_log2 = 22;
    uint32_t* hitmask = nullptr;
    uint32_t* tile_cnt = nullptr;
    uint32_t* grpsum = nullptr;
    // sharded training
    bool sharded = false;
    uint32_t rank = 0, world = 1;
    Table dt{};                    // per-merge count-delta table (local deltas before the exchange)
    uint32_t* d_nlog = nullptr;    // local length before each merge of a step
    uint32_t* h_nlog = nullptr;    // pinned
    uint32_t step_k = 0;
    uint32_t* rec_send = nullptr;  // exchange records of gbpe_shard_step_comm
    uint32_t* rec_recv = nullptr;
    uint64_t rec_words = 0;
    // stats
    uint64_t bytes_moved = 0;
    uint64_t max_live = 0;
    double ms_merge = 0, ms_select = 0, ms_other = 0, ms_delta = 0, ms_compact = 0;
    uint64_t timed_merges = 0;
    std::vector<hipEvent_t> evs;
    // sector-sparse loop
    bool sp = false;             // the stream is in the sector layout
    uint32_t sp_secw = 256;      // sector window (symbols)
    uint32_t max_id = 0;         // exclusive bound of every token id of the run (bitmap rows)
    uint32_t last_mc = 0;        // count of the last merge run
    int bcur = 0;                // dense buffer holding the body sectors
    uint32_t nsec = 0;
    uint64_t nsec_cap = 0, loc_cap = 0;
    uint32_t bend = 0;           // end of the body's sector windows in the body buffer
    uint32_t sp_shrinks = 0;     // zone shrinks since the last entry
    uint2* sec = nullptr;        // {start, count} per sector
    uint32_t* sp_loc = nullptr;  // per-sector scratch (starts / scan)
    uint64_t* sp_blk = nullptr;  // scan block totals
    uint32_t* bits = nullptr;    // presence bitmap, rows = token ids, W words per row
    uint32_t* sig = nullptr;     // per-sector pair signatures (SP_SIGW words each)
    uint64_t sig_cap = 0;
    uint64_t sp_age = 0;         // sparse merges since the signatures were built
    uint64_t sp_bits_age = 0;    // ... since the token bitmap was built
    uint64_t bits_cap = 0;       // words
    uint32_t W = 0;
    void* zbuf[2] = {nullptr, nullptr};
    void* wtmp = nullptr;        // stale-window source copy
    uint64_t zcap = 0;           // zone buffer capacity (symbols)
    int zcur = 0;                // zone buffer holding the zone
    DevState* zst = nullptr;     // the zone's loop state
    DevState* h_zst = nullptr;   // pinned
    uint32_t* d_u32 = nullptr;   // small device scratch
    uint64_t* part = nullptr;    // k_refresh workgroup maxima (sparse selection)
    uint32_t* zseg = nullptr;    // ZSegState: the zone segments' per-merge hand-off (k_refresh zeroes it)
    uint32_t zseg_mode = 1;      // GBPE_ZONE_SEG: 1 = segments for zones beyond zone_one (up to 1M), 0 = off
    uint32_t table_grows = 0;    // crowded-table rebuilds (same size or larger)
    uint64_t* wg_bytes = nullptr;   // bytes moved per k_body workgroup (each its own counter)
    uint32_t delta_mt = 2048;       // dense k_delta: multi-tile workgroups from this many tiles (0 = never; GBPE_DELTA_MT)
    uint32_t delta_tpw = 8;         // ... of 8, 16 or 32 tiles (GBPE_DELTA_TPW)
    uint64_t wg_cap = 0;
    double ms_sparse = 0, ms_dense = 0;   // GBPE_TRAIN_TIMING: merge passes (without selection / refresh) by mode
    double ms_body = 0;          // GBPE_TRAIN_TIMING: k_body alone
    uint64_t dense_bytes = 0;    // algorithmic stream bytes of the dense merges
    uint32_t g_refresh = 0;
    uint64_t sp_merges = 0, sp_sectors = 0, sp_zone = 0;
    uint32_t sp_enters = 0, sp_exits = 0;
    uint32_t sp_div = 64;        // enter when last_mc * sp_div <= n
    uint32_t sp_cooldown = 0;    // steps to stay dense after an abort
    uint32_t lx_div = 16;        // with the lexicon: enter once next_mc * lx_div <= n, from the first step on (GBPE_LEXICON_DIV)
    uint32_t sub_zone = 1u << 20;   // sparse steps run in sub-steps of sub_k merges while the zone exceeds this
    uint32_t sub_k = 16;            // (the zone shrinks between them; GBPE_SUBSTEP_ZONE, GBPE_SUBSTEP)
    bool zone16 = true;             // u16 zones of 8K-16K symbols: the 16-per-thread zone pass (GBPE_ZONE16=0: off)
    // persistent tail loop (k_tail)
    bool tail_on = true;         // GBPE_TAIL=0: never (a -DGBPE_TAIL_LOOP build only; measured no faster)
    uint32_t tail_mc = 4096;     // run a step in k_tail once the last count is at most this (GBPE_TAIL_MC)
    bool tail_skip = false;      // k_tail left the last step early: the next one runs k_body
    uint32_t* d_tstat = nullptr;
    uint64_t tail_merges = 0, tail_steps = 0, tail_exits = 0;
    double ms_tail = 0;
    uint32_t sp_zt = 5;          // zone target = sp_zt * last_mc + 64 (>= zone_f; GBPE_SPARSE_ZT; 4/5/6/7 measured
                                 // 0.895/0.893/0.918/0.918 s at 1 GiB with zone_f 3)
    uint32_t shrink_pct = 200;   // shrink once the zone exceeds shrink_pct % of the target + 4096 (GBPE_SHRINK_PCT)
    uint32_t zone_f = 3;         // single-GPU zone rule factor (sel_inline; GBPE_ZONE_F, >= 3)
    uint32_t refresh_blocks = 0; // GBPE_REFRESH_BLOCKS: k_refresh grid (0 = 2 per CU)
    bool rehash_on = true;       // GBPE_REHASH: grow the table inside the sparse loop (0: exit, grow, recount)
    uint32_t body_cap = 256;     // GBPE_BODY_WG: most k_body workgroups (default one per CU)
    uint32_t* d_clog = nullptr;  // GBPE_SPARSE_TRACE: per-merge candidate / hit sectors
    uint32_t* h_clog = nullptr;
    FILE* trace = nullptr;
    // word-lexicon body (lexicon.h): the sectors hold one copy of every
    // distinct body word instead of the body itself
    bool lex = false;            // the current sparse entry uses it
    bool lex_on = true;          // GBPE_LEXICON=0: never
    void* lx_store = nullptr;    // distinct words, each followed by a 0 separator (S symbols)
    uint32_t* lx_mul = nullptr;  // per store symbol: its word's occurrences (0 = separator / padding)
    uint64_t lx_cap = 0, lx_len = 0;   // store symbols: capacity, used
    uint32_t* lx_occ = nullptr;  // body words in stream order: uid, or LX_LIT | symbol
    uint64_t lx_occ_cap = 0, lx_nocc = 0;
    uint32_t* lx_w0 = nullptr;   // first uid of each sector window
    uint32_t lx_nuid = 0, lx_uid_cap = 0;
    void* lx_tmp = nullptr;      // build / expansion scratch (grown, kept)
    uint64_t lx_tmp_bytes = 0;
    uint64_t lx_words = 0, lx_builds = 0, lx_fallbacks = 0;   // stats
};

namespace {

int tr_err(gbpe_trainer* t, int code, const char* msg) { return gbpe_set_error(t->ctx, code, "%s", msg); }

#define TR_HIP(t, call) GBPE_HIP((t)->ctx, call)

// the symbols the sparse kernels merge: the lexicon store, or the body sectors in place
inline void* sp_body(const gbpe_trainer* t) { return t->lex ? t->lx_store : t->buf[t->bcur]; }
inline uint32_t* sp_mul(const gbpe_trainer* t) { return t->lex ? t->lx_mul : nullptr; }
// the single-GPU selection's zone rule (sel_inline)
inline SelShard sel_single(const gbpe_trainer* t) {
    SelShard sh;
    sh.zf = t->zone_f;
    return sh;
}


uint32_t grid_persistent(const gbpe_ctx* ctx, uint64_t work_tiles, uint32_t per_cu) {
    uint64_t g = (uint64_t)(ctx->num_cu > 0 ? ctx->num_cu : 256) * per_cu;
    if (work_tiles < g) g = work_tiles;
    return (uint32_t)(g ? g : 1);
}
// a grid over argmax blocks: every workgroup owns at most 64 (one flag ballot)
uint32_t grid_blocks(const gbpe_ctx* ctx, uint32_t nblk, uint32_t per_cu) {
    return std::max<uint32_t>(grid_persistent(ctx, nblk, per_cu), (uint32_t)gbpe_div_up(nblk, 64));
}

// new (empty) table arrays of 2^lg slots; the caller recounts (table_rebuild)
int table_resize(gbpe_trainer* t, uint32_t lg) {
    hipStream_t s = t->ctx->stream;
    TR_HIP(t, hipStreamSynchronize(s));
    hipFree(t->tb.slots);
    hipFree(t->tb.bmax);
    hipFree(t->tb.dirty);
    hipFree(t->tb.dlist);
    hipFree(t->tb.blive);
    t->tb.slots = nullptr, t->tb.bmax = nullptr, t->tb.dirty = nullptr, t->tb.dlist = nullptr, t->tb.blive = nullptr;
    const uint64_t slots = 1ull << lg;
    t->table_log2 = lg;
    t->tb.mask = (uint32_t)(slots - 1);
    t->tb.nblk = (uint32_t)(slots >> BLK_LOG2);
    if (hipMalloc(&t->tb.slots, slots * sizeof(uint2)) != hipSuccess ||
        hipMalloc(&t->tb.bmax, t->tb.nblk * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&t->tb.dirty, t->tb.nblk * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->tb.dlist, (t->tb.nblk + 1) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->tb.blive, t->tb.nblk * sizeof(uint32_t)) != hipSuccess)
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(pair table, 2^%u slots) failed", lg);
    TR_HIP(t, hipMemsetAsync(t->tb.dirty, 0, t->tb.nblk * sizeof(uint32_t), s));
    t->g_refresh = grid_blocks(t->ctx, t->tb.nblk, 2);
    if (t->refresh_blocks) t->g_refresh = std::max<uint32_t>(t->refresh_blocks, (uint32_t)gbpe_div_up(t->tb.nblk, 64));
    if (t->part) {   // one partial maximum per k_refresh workgroup
        hipFree(t->part);
        t->part = nullptr;
        TR_HIP(t, hipMalloc(&t->part, (uint64_t)(t->tb.nblk + 1) * sizeof(uint64_t)));
    }
    return GBPE_OK;
}

int table_rebuild(gbpe_trainer* t) {
    hipStream_t s = t->ctx->stream;
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    TR_HIP(t, hipMemsetAsync(t->tb.slots, 0, slots * sizeof(uint2), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.blive, 0, (uint64_t)t->tb.nblk * sizeof(uint32_t), s));
    TR_HIP(t, hipMemsetAsync(&t->st->used, 0, sizeof(uint32_t), s));
    const uint64_t ntiles = gbpe_div_up(t->n, TILE);
    const uint32_t g = grid_persistent(t->ctx, ntiles, 2);
    if (t->u16)
        hipLaunchKernelGGL(k_count_full<uint16_t>, dim3(g), dim3(TPB), 0, s, t->st,
                           (const uint16_t*)t->buf[t->cur], t->tb);
    else
        hipLaunchKernelGGL(k_count_full<uint32_t>, dim3(g), dim3(TPB), 0, s, t->st,
                           (const uint32_t*)t->buf[t->cur], t->tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    hipLaunchKernelGGL(k_clear_dirty_all, dim3(gbpe_div_up(t->tb.nblk, 256)), dim3(256), 0, s, t->st, t->tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    if (t->u16)
        hipLaunchKernelGGL(k_refresh<uint16_t>, dim3(grid_blocks(t->ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st, 0u,
                           0, t->tb, (uint16_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    else
        hipLaunchKernelGGL(k_refresh<uint32_t>, dim3(grid_blocks(t->ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st, 0u,
                           0, t->tb, (uint32_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

// Growing the table inside the sector-sparse loop: every count in the table is
// exact between steps (the body's multiplicities included), so the live entries
// move to the larger table as they are — no exit to one dense stream, no recount
// and no lexicon rebuild on re-entry (C5 grew 2^20 -> 2^25 in five such exits).
__global__ __launch_bounds__(TPB) void k_rehash(const uint2* __restrict__ old, uint64_t nold, DevState* st, Table tb) {
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i < nold; i += (uint64_t)gridDim.x * TPB) {
        const uint2 e = old[i];
        if (e.x && (int32_t)e.y > 0) table_add(tb, st, e.x, e.y);
    }
}

int table_rehash(gbpe_trainer* t, uint32_t lg) {
    hipStream_t s = t->ctx->stream;
    uint2* old = t->tb.slots;
    const uint64_t nold = (uint64_t)t->tb.mask + 1;
    t->tb.slots = nullptr;   // kept until the live entries have moved
    int rc = table_resize(t, lg);
    if (rc != GBPE_OK) {
        hipFree(old);
        return rc;
    }
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    TR_HIP(t, hipMemsetAsync(t->tb.slots, 0, slots * sizeof(uint2), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.blive, 0, (uint64_t)t->tb.nblk * sizeof(uint32_t), s));
    TR_HIP(t, hipMemsetAsync(&t->st->used, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_rehash, dim3(grid_persistent(t->ctx, gbpe_div_up(nold, TPB), 4)), dim3(TPB), 0, s,
                       (const uint2*)old, nold, t->st, t->tb);
    GBPE_LAUNCH_CHECK(t->ctx);
    hipLaunchKernelGGL(k_clear_dirty_all, dim3(gbpe_div_up(t->tb.nblk, 256)), dim3(256), 0, s, t->st, t->tb);
    // block maxima and the per-workgroup partial maxima the next selection reads
    if (t->u16)
        hipLaunchKernelGGL(k_refresh<uint16_t>, dim3(t->g_refresh), dim3(TPB), 0, s, t->st, 0u, 0, t->tb,
                           (uint16_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr,
                           FusedSel(), t->part, (uint32_t*)nullptr);
    else
        hipLaunchKernelGGL(k_refresh<uint32_t>, dim3(t->g_refresh), dim3(TPB), 0, s, t->st, 0u, 0, t->tb,
                           (uint32_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr,
                           FusedSel(), t->part, (uint32_t*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    TR_HIP(t, hipStreamSynchronize(s));
    hipFree(old);
    return GBPE_OK;
}

template <typename S>
int launch_merge(gbpe_trainer* t, uint32_t round, hipStream_t s, uint32_t g_delta, uint32_t g_compact,
                 uint32_t g_refresh, bool timing, hipEvent_t* ev) {
    S* cur = (S*)t->buf[t->cur ^ (round & 1)];
    S* oth = (S*)t->buf[t->cur ^ (round & 1) ^ 1];
    const bool exact = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) != 0;
    if (timing) TR_HIP(t, hipEventRecord(ev[0], s));
    hipLaunchKernelGGL(k_select, dim3(1), dim3(SEL_THREADS), 0, s, t->st, t->tb, t->d_log, t->grpsum,
                           (uint32_t*)nullptr, (uint32_t*)nullptr, (DevState*)nullptr, exact ? 1u : 0u);
    if (timing) TR_HIP(t, hipEventRecord(ev[1], s));
    // many tiles: TPW tiles per k_delta workgroup (fewer hot-pair flushes)
    const bool mt = t->delta_mt && g_delta >= t->delta_mt;
    const uint32_t tpw = t->delta_tpw;
    const uint32_t g_mt = (uint32_t)gbpe_div_up(g_delta, tpw);
    // stale-tail blocks (reference compaction): ~2K symbols each of the largest
    // possible tail (n/2), at most 1024
    const uint32_t g_mtail = exact ? 0u : (uint32_t)std::min<uint64_t>(1024, gbpe_div_up((uint64_t)t->n / 2 + 1, 2048));
    // the single-tile k_delta's tail blocks (1024-slot LDS table: ~1K-symbol slices)
    const uint32_t g_dtail = exact ? 0u : (uint32_t)std::min<uint64_t>(1024, gbpe_div_up((uint64_t)t->n / 2 + 1, 1024));
    if (exact) {
        if (mt)
            hipLaunchKernelGGL(tpw == 32 ? (k_delta_mt<S, true, 32>) : tpw == 16 ? (k_delta_mt<S, true, 16>) : (k_delta_mt<S, true, 8>),
                               dim3(g_mt + g_mtail), dim3(TPB), 0, s, t->st, round, (const S*)cur, t->tb, t->hitmask,
                               t->tile_cnt, t->grpsum, g_delta, g_mt);
        else
            hipLaunchKernelGGL((k_delta<S, true>), dim3(g_delta), dim3(TPB), 0, s, t->st, round, (const S*)cur, t->tb,
                               t->hitmask, t->tile_cnt, t->grpsum, g_delta, 0xFFFFFFFFu);
        if (timing) TR_HIP(t, hipEventRecord(ev[3], s));
        hipLaunchKernelGGL((k_compact<S, true>), dim3(g_compact), dim3(CTPB), 0, s, t->st, round, cur, oth,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb);
    } else {
        if (mt)
            hipLaunchKernelGGL(tpw == 32 ? (k_delta_mt<S, false, 32>) : tpw == 16 ? (k_delta_mt<S, false, 16>) : (k_delta_mt<S, false, 8>),
                               dim3(g_mt + g_mtail), dim3(TPB), 0, s, t->st, round, (const S*)cur, t->tb, t->hitmask,
                               t->tile_cnt, t->grpsum, g_delta, g_mt);
        else
            hipLaunchKernelGGL((k_delta<S, false>), dim3(g_delta + g_dtail), dim3(TPB), 0, s, t->st, round, (const S*)cur,
                               t->tb, t->hitmask, t->tile_cnt, t->grpsum, g_delta, g_delta);
        if (timing) TR_HIP(t, hipEventRecord(ev[3], s));
        hipLaunchKernelGGL((k_compact<S, false>), dim3(g_compact), dim3(CTPB), 0, s, t->st, round, cur, oth,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb);
    }
    if (timing) TR_HIP(t, hipEventRecord(ev[2], s));
    FusedSel fs;
    fs.log = nullptr;
    fs.grpsum = t->grpsum;
    fs.exact = exact ? 1u : 0u;
    hipLaunchKernelGGL(k_refresh<S>, dim3(g_refresh), dim3(TPB), 0, s, t->st, round, 1, t->tb, cur,
                       (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, fs);
    if (timing) TR_HIP(t, hipEventRecord(ev[4], s));
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

// ── sector-sparse loop: launches and re-layouts ──

struct SpGrid {
    uint32_t body, copy, zdelta, zcompact, refresh;
    uint32_t wpg = 16;    // bitmap words per k_body workgroup
    uint32_t ztail = 0;   // stale-tail slice blocks of the multi-tile zone k_delta
    uint32_t zone1;   // zone workgroups inside k_body: 1 = zone_one, >= 2 = zone_seg segments, 0 = multi-tile passes
    int bt;       // k_body workgroup size (256 or 1024)
};

template <typename S>
uint32_t zone_max(int bt) {
    return bt == 1023 ? 1024u * 16u : bt == 1024 ? ZoneDim<S, 1024>::ZMAX : ZoneDim<S, 256>::ZMAX;
}
// k_body grid: bitmap words per workgroup (>= the measured best 16 / 32 at C2 size),
// at most `cap` workgroups (GBPE_BODY_WG; default 4 per CU)
inline void body_grid(const gbpe_trainer* t, int bt, uint32_t* nbody, uint32_t* wpg) {
    const uint32_t W = (uint32_t)gbpe_div_up(t->nsec, 32);
    const uint32_t minw = bt == 1024 ? 32u : 16u;
    uint32_t g = (uint32_t)gbpe_div_up(W, minw);
    if (g > t->body_cap) g = t->body_cap;
    if (g == 0) g = 1;
    *wpg = (uint32_t)gbpe_div_up(W, g);
    if (*wpg == 0) *wpg = 1;
    *nbody = (uint32_t)gbpe_div_up(W, *wpg);
    if (*nbody == 0) *nbody = 1;
}

// launch k_body<S, EXACT, bt> (one instantiation per workgroup size)
// bt: 256, 1024, or 1023 = 1024 threads with 16 zone symbols each (u16 zones of
// 8K-16K symbols: half the per-thread zone work of the 32K form; 1 GiB en1g
// 1.017 -> 0.963 s.  1024 threads x 8 for zones <= 8K instead of 256 x 32 was
// slower: C2 0.66 vs 0.61 s)
template <typename S, bool EXACT, typename... A>
void launch_body(int bt, uint32_t grid, hipStream_t s, A... args) {
    if (bt == 2048)   // zone segments inside k_body (the ZSEG form, 1024 threads)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024, 16, true>), dim3(grid), dim3(1024), 0, s, args...);
    else if (bt == 1023 && sizeof(S) == 2)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024, 16>), dim3(grid), dim3(1024), 0, s, args...);
    else if (bt >= 1023)
        hipLaunchKernelGGL((k_body<S, EXACT, 1024>), dim3(grid), dim3(1024), 0, s, args...);
    else
        hipLaunchKernelGGL((k_body<S, EXACT, 256>), dim3(grid), dim3(256), 0, s, args...);
}

template <typename S>
int launch_merge_sparse(gbpe_trainer* t, uint32_t round, hipStream_t s, const SpGrid& g, bool timing, hipEvent_t* ev) {
    S* zc = (S*)t->zbuf[t->zcur ^ (round & 1)];
    S* zo = (S*)t->zbuf[t->zcur ^ (round & 1) ^ 1];
    const bool exact = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) != 0;
    if (timing) TR_HIP(t, hipEventRecord(ev[0], s));
    if (timing) TR_HIP(t, hipEventRecord(ev[1], s));   // selection runs inside k_body (sel_inline)
    // zone segments run inside k_body (its ZSEG form)
    const bool inbody = g.zone1 >= 2;
    const uint32_t gb = g.body + (g.zone1 ? g.zone1 : g.copy);
    const uint32_t z1 = g.zone1;   // k_body's own zone workgroups
    const int bt = inbody ? 2048 : g.bt;
    // events: [1] k_body [3] zone k_delta + k_compact (multi-tile zone) [2] k_refresh [4]
    if (exact)
        launch_body<S, true>(bt, gb, s, t->st, round, (S*)sp_body(t), t->sec, t->bits, t->W, g.wpg, t->sig, t->tb,
                             g.body, (const S*)zo, (S*)t->wtmp, t->d_clog ? 1u : 0u, t->zst, zc, z1,
                             (const uint64_t*)t->part, g.refresh, t->d_log, t->grpsum, t->wg_bytes, t->tb, sel_single(t),
                             sp_mul(t), (ZSegState*)t->zseg);
    else
        launch_body<S, false>(bt, gb, s, t->st, round, (S*)sp_body(t), t->sec, t->bits, t->W, g.wpg, t->sig, t->tb,
                              g.body, (const S*)zo, (S*)t->wtmp, t->d_clog ? 1u : 0u, t->zst, zc, z1,
                              (const uint64_t*)t->part, g.refresh, t->d_log, t->grpsum, t->wg_bytes, t->tb, sel_single(t),
                             sp_mul(t), (ZSegState*)t->zseg);
    if (timing) TR_HIP(t, hipEventRecord(ev[3], s));
    if (!g.zone1) {
        // a zone of many tiles (the lexicon loop's first merges): TPW tiles per
        // workgroup and one flush of their hot pairs, as in the dense loop
        const bool mt = t->delta_mt && g.zdelta >= t->delta_mt;
        const uint32_t g_mt = (uint32_t)gbpe_div_up(g.zdelta, 8);
        if (exact && mt)
            hipLaunchKernelGGL((k_delta_mt<S, true, 8>), dim3(g_mt), dim3(TPB), 0, s, t->zst, round, (const S*)zc, t->tb,
                               t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g_mt);
        else if (mt)
            hipLaunchKernelGGL((k_delta_mt<S, false, 8>), dim3(g_mt + g.ztail), dim3(TPB), 0, s, t->zst, round,
                               (const S*)zc, t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g_mt);
        else if (exact)
            hipLaunchKernelGGL((k_delta<S, true, true>), dim3(g.zdelta), dim3(TPB), 0, s, t->zst, round, (const S*)zc,
                               t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, 0xFFFFFFFFu);
        else   // + stale-tail slice blocks: the zone's tail (<= mc <= zone/5) in ~2K-symbol slices
            hipLaunchKernelGGL((k_delta<S, false, true>), dim3(g.zdelta + g.ztail), dim3(TPB), 0, s, t->zst, round,
                               (const S*)zc, t->tb, t->hitmask, t->tile_cnt, t->grpsum, g.zdelta, g.zdelta);
    }
    if (!g.zone1) {
        if (exact)
            hipLaunchKernelGGL((k_compact<S, true, true>), dim3(g.zcompact), dim3(CTPB), 0, s, t->zst, round, zc, zo,
                               (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum,
                               t->tb, (const S*)t->wtmp, (const DevState*)t->st);
        else
            hipLaunchKernelGGL((k_compact<S, false, true>), dim3(g.zcompact), dim3(CTPB), 0, s, t->zst, round, zc, zo,
                               (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum,
                               t->tb, (const S*)t->wtmp, (const DevState*)t->st);
    }
    if (timing) TR_HIP(t, hipEventRecord(ev[2], s));
    hipLaunchKernelGGL(k_refresh<S>, dim3(g.refresh), dim3(TPB), 0, s, t->st, round, 2, t->tb, (S*)nullptr,
                       (const uint32_t*)nullptr, t->zst, t->d_clog, FusedSel(), t->part, t->zseg);
    if (timing) TR_HIP(t, hipEventRecord(ev[4], s));
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

template <typename T>
int sp_grow(gbpe_trainer* t, T** p, uint64_t* cap, uint64_t need) {
    if (*p && *cap >= need) return GBPE_OK;
    hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void**)p, need * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(sparse layout, %llu B) failed",
                              (unsigned long long)(need * sizeof(T)));
    }
    *cap = need;
    return GBPE_OK;
}

// sectors over body positions [base, base + len) appended after sector t->nsec
// (their token bits and signatures too); base is a word start
template <typename S>
int sp_add_sectors(gbpe_trainer* t, uint32_t base, uint32_t len) {
    hipStream_t s = t->ctx->stream;
    const uint32_t nw = (uint32_t)gbpe_div_up(len, t->sp_secw);
    if ((uint64_t)t->nsec + nw > t->nsec_cap || (uint64_t)t->nsec + nw > (uint64_t)t->W * 32 ||
        ((uint64_t)t->nsec + nw) * SP_SIGW > t->sig_cap || nw > t->loc_cap)
        return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "sector capacity exceeded");
    const S* body = (const S*)t->buf[t->bcur];
    hipLaunchKernelGGL(k_sp_sectors<S>, dim3((uint32_t)gbpe_div_up(nw, TPB / 64)), dim3(TPB), 0, s, body, base, len,
                       t->sp_secw, t->sp_loc, nw);
    hipLaunchKernelGGL(k_sp_sector_len, dim3((uint32_t)gbpe_div_up(nw, 256)), dim3(256), 0, s, (const uint32_t*)t->sp_loc,
                       nw, base + len, t->sec + t->nsec);
    if (t->nsec == 0) {   // a fresh build (sp_enter): whole columns
        hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(nw, TPB / 64)), dim3(TPB), 0, s, body,
                           (const uint2*)t->sec, 0u, nw, (uint32_t*)nullptr, t->W, t->sig);
        hipLaunchKernelGGL(k_sp_colbits<S>, dim3((uint32_t)gbpe_div_up(nw, 32)), dim3(TPB), 0, s, body,
                           (const uint2*)t->sec, nw, t->bits, t->W);
    } else {
        hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(nw, TPB / 64)), dim3(TPB), 0, s, body,
                           (const uint2*)t->sec, t->nsec, nw, t->bits, t->W, t->sig);
    }
    GBPE_LAUNCH_CHECK(t->ctx);
    t->nsec += nw;
    t->bend = base + len;
    return GBPE_OK;
}

// (re)build the pair signatures (and, with `with_bits`, the token bitmap) from the
// body sectors: stale entries make the filters looser, never wrong
template <typename S>
int sp_filters(gbpe_trainer* t, bool with_bits) {
    hipStream_t s = t->ctx->stream;
    hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(t->nsec, TPB / 64)), dim3(TPB), 0, s,
                       (const S*)sp_body(t), (const uint2*)t->sec, 0u, t->nsec, (uint32_t*)nullptr, t->W, t->sig);
    if (with_bits) {
        TR_HIP(t, hipMemsetAsync(t->bits, 0, (uint64_t)t->max_id * t->W * 4, s));
        hipLaunchKernelGGL(k_sp_colbits<S>, dim3((uint32_t)gbpe_div_up(t->nsec, 32)), dim3(TPB), 0, s,
                           (const S*)sp_body(t), (const uint2*)t->sec, t->nsec, t->bits, t->W);
    }
    GBPE_LAUNCH_CHECK(t->ctx);
    t->sp_age = 0;
    if (with_bits) t->sp_bits_age = 0;
    return GBPE_OK;
}

// ── word-lexicon body ──

// bump allocation over the trainer's lexicon scratch
struct LxCarve {
    char* base;
    uint64_t used = 0;
    template <typename T>
    T* take(uint64_t n) {
        const uint64_t b = (used + 255) & ~255ull;
        used = b + n * sizeof(T);
        return reinterpret_cast<T*>(base + b);
    }
};

int lx_scratch(gbpe_trainer* t, uint64_t bytes) {
    if (t->lx_tmp && t->lx_tmp_bytes >= bytes) return GBPE_OK;
    TR_HIP(t, hipStreamSynchronize(t->ctx->stream));
    hipFree(t->lx_tmp);
    t->lx_tmp = nullptr;
    t->lx_tmp_bytes = 0;
    if (hipMalloc(&t->lx_tmp, bytes) != hipSuccess) {
        t->lx_tmp = nullptr;
        return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(lexicon scratch, %llu B) failed", (unsigned long long)bytes);
    }
    t->lx_tmp_bytes = bytes;
    return GBPE_OK;
}

// exclusive scan of n u32 counts in place (k_chunk_scan1/2); blk gets n/SCAN_BLK + 2
// entries, the total at blk[nblk]
inline void lx_scan(hipStream_t s, uint32_t* v, uint64_t n, uint64_t* blk) {
    const uint64_t nb = gbpe_div_up(n ? n : 1, SCAN_BLK);
    hipLaunchKernelGGL(k_chunk_scan1, dim3((uint32_t)nb), dim3(SCAN_TPB), 0, s, (const uint32_t*)v, n, v, blk);
    hipLaunchKernelGGL(k_chunk_scan2, dim3(1), dim3(SCAN_TPB), 0, s, blk, nb, blk + nb);
}

// What a segment's words would add to the lexicon (nothing is committed yet)
struct LxPlan {
    bool ok = false;
    uint32_t nw = 0, nshort = 0, nlong = 0, nu = 0, T = 0;   // words, distinct short / long, entries, store symbols
    uint32_t *wpos = nullptr, *usz = nullptr, *umul = nullptr, *urep = nullptr, *occ = nullptr, *upre = nullptr;
    uint64_t* ublk = nullptr;
};

// Dedup the words of seg[0, len) (a word starts at 0): word starts, the word
// table, entries (uids from t->lx_nuid) and the segment's occurrence list, in
// the scratch.  plan.ok = false when a hash collision or a full word table
// makes the segment unusable, or (fresh) the store would not be much smaller
// than the segment.
template <typename S>
int lx_analyze(gbpe_trainer* t, const S* seg, uint32_t len, bool fresh, LxPlan& lp) {
    hipStream_t s = t->ctx->stream;
    lp = LxPlan();
    if (len == 0) return GBPE_OK;
    const uint64_t ntiles = gbpe_div_up(len, TILE);
    // word count first (sizes the rest of the scratch)
    int rc = lx_scratch(t, (ntiles + 64) * 4 + (ntiles / SCAN_BLK + 4) * 8 + 1024);
    if (rc != GBPE_OK) return rc;
    {
        LxCarve c{(char*)t->lx_tmp};
        uint32_t* tc = c.take<uint32_t>(ntiles);
        uint64_t* tb = c.take<uint64_t>(ntiles / SCAN_BLK + 4);
        hipLaunchKernelGGL(k_lx_count<S>, dim3((uint32_t)ntiles), dim3(TPB), 0, s, seg, len, tc);
        lx_scan(s, tc, ntiles, tb);
        GBPE_LAUNCH_CHECK(t->ctx);
        uint64_t nw64 = 0;
        TR_HIP(t, hipMemcpyAsync(&nw64, tb + gbpe_div_up(ntiles, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
        lp.nw = (uint32_t)nw64;
    }
    const uint32_t nw = lp.nw;
    uint64_t P = 4096;
    while (P < 2ull * nw && P < (1ull << 27)) P <<= 1;
    const uint64_t nbb = gbpe_div_up(P, LX_TB);
    const uint64_t need = (ntiles + 64) * 4 + (ntiles / SCAN_BLK + 4) * 8 + 9ull * (nw + 64) * 4 + P * 16 +
                          (nbb + 64) * 4 + 2 * (nbb / SCAN_BLK + (uint64_t)nw / SCAN_BLK + 8) * 8 + 32 * 256;
    rc = lx_scratch(t, need);
    if (rc != GBPE_OK) return rc;
    LxCarve c{(char*)t->lx_tmp};
    uint32_t* tc = c.take<uint32_t>(ntiles);
    uint64_t* tb = c.take<uint64_t>(ntiles / SCAN_BLK + 4);
    lp.wpos = c.take<uint32_t>(nw + 1);
    uint32_t* otmp = c.take<uint32_t>(nw + 1);
    uint32_t* longs = c.take<uint32_t>(nw + 1);
    lp.usz = c.take<uint32_t>(nw + 1);
    lp.umul = c.take<uint32_t>(nw + 1);
    lp.urep = c.take<uint32_t>(nw + 1);
    lp.occ = c.take<uint32_t>(nw + 1);
    auto* keys = c.take<unsigned long long>(P);
    auto* vals = c.take<uint2>(P);
    uint32_t* bc = c.take<uint32_t>(nbb);
    uint64_t* bb = c.take<uint64_t>(nbb / SCAN_BLK + 4);
    lp.ublk = c.take<uint64_t>((uint64_t)nw / SCAN_BLK + 4);
    uint32_t* ctr = c.take<uint32_t>(8);
    // (the tile counts are recomputed: the scratch may have moved)
    hipLaunchKernelGGL(k_lx_count<S>, dim3((uint32_t)ntiles), dim3(TPB), 0, s, seg, len, tc);
    lx_scan(s, tc, ntiles, tb);
    hipLaunchKernelGGL(k_lx_wpos<S>, dim3((uint32_t)ntiles), dim3(TPB), 0, s, seg, len, (const uint32_t*)tc,
                       (const uint64_t*)tb, lp.wpos);
    TR_HIP(t, hipMemsetAsync(keys, 0, P * 8, s));
    TR_HIP(t, hipMemsetAsync(vals, 0, P * 8, s));
    TR_HIP(t, hipMemsetAsync(ctr, 0, 32, s));
    if (nw)
        hipLaunchKernelGGL(k_lx_hash<S>, dim3((uint32_t)gbpe_div_up(nw, TPB * LX_WPT)), dim3(TPB), 0, s, seg, len,
                           (const uint32_t*)lp.wpos, nw, keys, vals, (uint32_t)P, otmp, longs, ctr);
    hipLaunchKernelGGL(k_lx_tabcount, dim3((uint32_t)nbb), dim3(TPB), 0, s, (const unsigned long long*)keys, (uint32_t)P, bc);
    lx_scan(s, bc, nbb, bb);
    GBPE_LAUNCH_CHECK(t->ctx);
    uint32_t h[4] = {0, 0, 0, 0};
    uint64_t nshort = 0;
    TR_HIP(t, hipMemcpyAsync(h, ctr, 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipMemcpyAsync(&nshort, bb + gbpe_div_up(nbb, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (h[1]) return GBPE_OK;   // word table overflow: not usable
    lp.nshort = (uint32_t)nshort;
    lp.nlong = h[0];
    lp.nu = lp.nshort + lp.nlong;
    if ((uint64_t)t->lx_nuid + lp.nu >= LX_LONG) return GBPE_OK;
    hipLaunchKernelGGL(k_lx_tabuid, dim3((uint32_t)nbb), dim3(TPB), 0, s, (const unsigned long long*)keys, vals, (uint32_t)P,
                       (const uint32_t*)bc, (const uint64_t*)bb, (const uint32_t*)lp.wpos, nw, len, lp.usz, lp.umul, lp.urep);
    if (lp.nlong)
        hipLaunchKernelGGL(k_lx_longs, dim3((uint32_t)gbpe_div_up(lp.nlong, 256)), dim3(256), 0, s, (const uint32_t*)longs,
                           (const uint32_t*)ctr, lp.nshort, (const uint32_t*)lp.wpos, nw, len, lp.usz, lp.umul, lp.urep);
    if (nw)
        hipLaunchKernelGGL(k_lx_occ<S>, dim3((uint32_t)gbpe_div_up(nw, 256)), dim3(256), 0, s, seg, (const uint32_t*)lp.wpos, nw,
                           len, (const uint32_t*)otmp, (const unsigned long long*)keys, (const uint2*)vals, (uint32_t)P,
                           (const uint32_t*)lp.urep, (const uint32_t*)lp.usz, lp.nshort, t->lx_nuid, lp.occ, ctr);
    // store offsets: exclusive scan of the entry sizes, in otmp (k_lx_occ, queued
    // before on the same stream, has consumed it)
    uint32_t* upre = otmp;
    TR_HIP(t, hipMemcpyAsync(upre, lp.usz, (uint64_t)lp.nu * 4, hipMemcpyDeviceToDevice, s));
    lx_scan(s, upre, lp.nu, lp.ublk);
    GBPE_LAUNCH_CHECK(t->ctx);
    uint64_t T = 0;
    TR_HIP(t, hipMemcpyAsync(&T, lp.ublk + gbpe_div_up(lp.nu ? lp.nu : 1, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipMemcpyAsync(h, ctr, 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (h[1]) return GBPE_OK;   // a hash collision (or a word missing from the table)
    lp.T = (uint32_t)T;
    if (fresh && T * 2 > len) return GBPE_OK;   // not worth it: the store would be more than half the body
    lp.upre = upre;
    lp.ok = true;
    return GBPE_OK;
}

// Append a planned segment to the lexicon: store entries (window-aligned), their
// sector windows after t->nsec with token bits and signatures, occurrences after
// t->lx_nocc.  plan.ok = false (nothing changed) when the capacities cannot take it.
template <typename S>
int lx_commit(gbpe_trainer* t, LxPlan& lp, const S* seg, bool fresh) {
    hipStream_t s = t->ctx->stream;
    const uint32_t SEC = t->sp_secw;
    const uint64_t sbase = gbpe_div_up(t->lx_len, SEC) * SEC;
    const uint64_t nwin = gbpe_div_up(lp.T ? lp.T : 1, SEC);
    const uint64_t kb = sbase / SEC;
    if (sbase + nwin * SEC > t->lx_cap || kb + nwin > t->nsec_cap || kb + nwin > (uint64_t)t->W * 32 ||
        (kb + nwin) * SP_SIGW > t->sig_cap || nwin > t->loc_cap || t->lx_nocc + lp.nw > t->lx_occ_cap) {
        lp.ok = false;
        return GBPE_OK;
    }
    S* store = (S*)t->lx_store;
    if (sbase > t->lx_len) {   // alignment padding: separators no sector covers
        TR_HIP(t, hipMemsetAsync(store + t->lx_len, 0, (sbase - t->lx_len) * sizeof(S), s));
        TR_HIP(t, hipMemsetAsync(t->lx_mul + t->lx_len, 0, (sbase - t->lx_len) * 4, s));
    }
    const uint32_t* upre = lp.upre;
    if (lp.nu) {
        hipLaunchKernelGGL(k_lx_fill<S>, dim3((uint32_t)gbpe_div_up(lp.nu, 256)), dim3(256), 0, s, seg,
                           (const uint32_t*)lp.urep, (const uint32_t*)lp.usz, (const uint32_t*)lp.umul, upre,
                           (const uint64_t*)lp.ublk, lp.nu, store + sbase, t->lx_mul + sbase);
        TR_HIP(t, hipMemsetAsync(t->sp_loc, 0xFF, nwin * 4, s));
        hipLaunchKernelGGL(k_lx_secstart, dim3((uint32_t)gbpe_div_up(lp.nu, 256)), dim3(256), 0, s, upre,
                           (const uint64_t*)lp.ublk, lp.nu, SEC, (uint32_t)sbase, t->lx_nuid, t->sp_loc, t->lx_w0 + kb);
        hipLaunchKernelGGL(k_sp_sector_len, dim3((uint32_t)gbpe_div_up(nwin, 256)), dim3(256), 0, s,
                           (const uint32_t*)t->sp_loc, (uint32_t)nwin, (uint32_t)(sbase + lp.T), t->sec + kb);
    } else {
        TR_HIP(t, hipMemsetAsync(t->sec + kb, 0, nwin * sizeof(uint2), s));
    }
    if (lp.nw)
        TR_HIP(t, hipMemcpyAsync(t->lx_occ + t->lx_nocc, lp.occ, (uint64_t)lp.nw * 4, hipMemcpyDeviceToDevice, s));
    // token bits and signatures of the new sectors (a fresh build: whole columns)
    hipLaunchKernelGGL(k_sp_bits<S>, dim3((uint32_t)gbpe_div_up(nwin, TPB / 64)), dim3(TPB), 0, s, (const S*)store,
                       (const uint2*)t->sec, (uint32_t)kb, (uint32_t)nwin, fresh ? (uint32_t*)nullptr : t->bits, t->W, t->sig);
    if (fresh)
        hipLaunchKernelGGL(k_sp_colbits<S>, dim3((uint32_t)gbpe_div_up(nwin, 32)), dim3(TPB), 0, s, (const S*)store,
                           (const uint2*)t->sec, (uint32_t)nwin, t->bits, t->W);
    GBPE_LAUNCH_CHECK(t->ctx);
    t->nsec = (uint32_t)(kb + nwin);
    t->lx_len = sbase + lp.T;
    t->lx_nocc += lp.nw;
    t->lx_nuid += lp.nu;
    t->lx_words += lp.nw;
    return GBPE_OK;
}

// lexicon → dense stream: every body word occurrence's current symbols, in
// stream order, to dst[0, B); returns the symbol total through *tot
template <typename S>
int lx_expand(gbpe_trainer* t, S* dst, uint64_t* tot) {
    hipStream_t s = t->ctx->stream;
    const uint64_t nu = t->lx_nuid, no = t->lx_nocc;
    int rc = lx_scratch(t, (2 * nu + no + 64) * 4 + (no / SCAN_BLK + 8) * 8 + 4096);
    if (rc != GBPE_OK) return rc;
    LxCarve c{(char*)t->lx_tmp};
    uint32_t* coff = c.take<uint32_t>(nu + 1);
    uint32_t* clen = c.take<uint32_t>(nu + 1);
    uint32_t* olen = c.take<uint32_t>(no + 1);
    uint64_t* oblk = c.take<uint64_t>(no / SCAN_BLK + 4);
    if (t->nsec)
        hipLaunchKernelGGL(k_lx_wordpos<S>, dim3((uint32_t)gbpe_div_up(t->nsec, TPB / 64)), dim3(TPB), 0, s,
                           (const S*)t->lx_store, (const uint2*)t->sec, t->nsec, (const uint32_t*)t->lx_w0, coff, clen);
    if (no)
        hipLaunchKernelGGL(k_lx_olen, dim3((uint32_t)gbpe_div_up(no, 256)), dim3(256), 0, s, (const uint32_t*)t->lx_occ, no,
                           (const uint32_t*)clen, olen);
    lx_scan(s, olen, no, oblk);
    if (no)
        hipLaunchKernelGGL(k_lx_expand<S>, dim3((uint32_t)gbpe_div_up(no, 256)), dim3(256), 0, s, (const uint32_t*)t->lx_occ,
                           no, (const uint32_t*)coff, (const uint32_t*)clen, (const S*)t->lx_store, (const uint32_t*)olen,
                           (const uint64_t*)oblk, dst);
    GBPE_LAUNCH_CHECK(t->ctx);
    TR_HIP(t, hipMemcpyAsync(tot, oblk + gbpe_div_up(no ? no : 1, SCAN_BLK), 8, hipMemcpyDeviceToHost, s));
    return GBPE_OK;
}

// dense → sparse at a step boundary.  The zone is the stream from the last word
// start at or before n - zt (zt = max(sp_zt * next_mc, 2 next_mc + last_mc) + 64:
// >= 5 x the next merge's count while counts fall, and room for the stale window
// the last merge left (sel_inline's zone rule); a merge that would not fit is not
// run and the host goes dense, sp_abort); the dense stale buffer's tail becomes the
// zone's stale buffer.  next_mc = 0: the last merge's count stands in for it.
template <typename S>
int sp_enter(gbpe_trainer* t, bool with_zone = true, uint32_t next_mc = 0) {
    hipStream_t s = t->ctx->stream;
    const uint32_t n = t->n;
    const uint64_t prev_mc = t->last_mc;   // the previous stream is n + prev_mc long
    const uint64_t nmc = next_mc ? next_mc : prev_mc;
    const uint64_t zt = std::max<uint64_t>((uint64_t)t->sp_zt * nmc, 2ull * nmc + prev_mc) + 64;
    const S* cur = (const S*)t->buf[t->cur];
    const S* stale = (const S*)t->buf[t->cur ^ 1];
    if (!t->d_u32) TR_HIP(t, hipMalloc(&t->d_u32, 64));
    uint32_t Zs = n;   // sharded ranks before the last: all body, no zone
    if (with_zone) {
        if (zt + 2 >= n) return GBPE_OK;
        hipLaunchKernelGGL(k_sp_zone_start<S>, dim3(1), dim3(1024), 0, s, cur, (uint32_t)(n - zt), t->d_u32);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipMemcpyAsync(&Zs, t->d_u32, 4, hipMemcpyDeviceToHost, s));
        TR_HIP(t, hipStreamSynchronize(s));
        if (Zs < t->sp_secw) return GBPE_OK;   // the whole stream is one long word (or tiny): stay dense
    }
    const uint32_t z = n - Zs;
    // word lexicon: plan the deduplicated body first; it sizes the sectors
    t->lex = false;
    t->lx_len = t->lx_nocc = 0;
    t->lx_nuid = 0;
    LxPlan lp;
    if (t->lex_on && Zs) {
        int rc0 = lx_analyze<S>(t, cur, Zs, true, lp);
        if (rc0 != GBPE_OK) return rc0;
        if (lp.ok) ++t->lx_builds;
        else ++t->lx_fallbacks;
    }
    // capacities for every sector the body can ever hold: windows over [0, n) (the
    // lexicon: over its store, and twice the zone for the words shrinks append) plus
    // one partial window per zone shrink (at most SP_SHRINKS per entry)
    const uint64_t cap = lp.ok ? gbpe_div_up((uint64_t)lp.T + 2ull * z, t->sp_secw) + 2 * (SP_SHRINKS + 1)
                               : gbpe_div_up(n, t->sp_secw) + SP_SHRINKS + 1;
    int rc = sp_grow(t, &t->sec, &t->nsec_cap, cap);
    if (rc == GBPE_OK && (!t->sp_loc || t->loc_cap < cap)) {
        hipFree(t->sp_loc);
        hipFree(t->sp_blk);
        t->sp_loc = nullptr;
        t->sp_blk = nullptr;
        t->loc_cap = 0;
        if (hipMalloc(&t->sp_loc, cap * 4) != hipSuccess ||
            hipMalloc(&t->sp_blk, (gbpe_div_up(cap, SCAN_BLK) + 1) * 8) != hipSuccess)
            rc = gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(sector scratch) failed");
        else
            t->loc_cap = cap;
    }
    if (rc != GBPE_OK) return rc;
    t->W = (uint32_t)gbpe_div_up(cap, 32);
    rc = sp_grow(t, &t->bits, &t->bits_cap, (uint64_t)t->max_id * t->W);
    if (rc == GBPE_OK) rc = sp_grow(t, &t->sig, &t->sig_cap, cap * SP_SIGW);
    if (rc != GBPE_OK) return rc;
    t->bcur = t->cur;
    t->nsec = 0;
    TR_HIP(t, hipMemsetAsync(t->bits, 0, (uint64_t)t->max_id * t->W * 4, s));
    TR_HIP(t, hipMemsetAsync(t->sig, 0, cap * SP_SIGW * 4, s));
    if (lp.ok) {
        const uint64_t scap = cap * t->sp_secw, ocap = (uint64_t)lp.nw + z + 1;
        if (!t->lx_store || t->lx_cap < scap) {
            hipFree(t->lx_store);
            hipFree(t->lx_mul);
            hipFree(t->lx_w0);
            t->lx_store = nullptr;
            t->lx_mul = t->lx_w0 = nullptr;
            t->lx_cap = 0;
            if (hipMalloc(&t->lx_store, scap * t->bps) != hipSuccess || hipMalloc(&t->lx_mul, scap * 4) != hipSuccess ||
                hipMalloc(&t->lx_w0, cap * 4) != hipSuccess)
                return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(word lexicon) failed");
            t->lx_cap = scap;
        }
        rc = sp_grow(t, &t->lx_occ, &t->lx_occ_cap, ocap);
        if (rc != GBPE_OK) return rc;
        t->lex = true;
        rc = lx_commit<S>(t, lp, cur, true);
        if (rc == GBPE_OK && !lp.ok) rc = gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "word lexicon capacity");
        if (rc == GBPE_OK && getenv("GBPE_LEX_CHECK")) {   // diagnostic: the lexicon expands back to the body
            S* chk = nullptr;
            TR_HIP(t, hipMalloc(&chk, ((uint64_t)Zs + 64) * sizeof(S)));
            uint64_t tot = 0;
            rc = lx_expand<S>(t, chk, &tot);
            std::vector<S> a(Zs), b(Zs);
            TR_HIP(t, hipStreamSynchronize(s));
            TR_HIP(t, hipMemcpy(a.data(), chk, (uint64_t)Zs * sizeof(S), hipMemcpyDeviceToHost));
            TR_HIP(t, hipMemcpy(b.data(), cur, (uint64_t)Zs * sizeof(S), hipMemcpyDeviceToHost));
            hipFree(chk);
            uint64_t bad = Zs;
            for (uint64_t i = 0; i < Zs; ++i)
                if (a[i] != b[i]) {
                    bad = i;
                    break;
                }
            std::vector<uint32_t> mm(lp.T);
            std::vector<S> ss(lp.T);
            TR_HIP(t, hipMemcpy(mm.data(), t->lx_mul, (uint64_t)lp.T * 4, hipMemcpyDeviceToHost));
            TR_HIP(t, hipMemcpy(ss.data(), t->lx_store, (uint64_t)lp.T * sizeof(S), hipMemcpyDeviceToHost));
            uint64_t wsum = 0, nz = 0, badm = 0;
            for (uint32_t i = 0; i < lp.T; ++i) {
                wsum += mm[i];
                if ((ss[i] == 0) != (mm[i] == 0)) ++badm;
            }
            for (uint32_t i = 0; i < Zs; ++i) nz += (b[i] & Sym<S>::TM) ? 1 : 0;
            fprintf(stderr, "[lex-check] Zs=%u words=%u distinct=%u+%u store=%u expanded=%llu first_diff=%llu "
                    "mult_sum=%llu nonzero_body=%llu sep_mismatch=%llu\n", Zs, lp.nw,
                    lp.nshort, lp.nlong, lp.T, (unsigned long long)tot, (unsigned long long)bad,
                    (unsigned long long)wsum, (unsigned long long)nz, (unsigned long long)badm);
        }
    } else {
        rc = sp_add_sectors<S>(t, 0u, Zs);
    }
    if (rc != GBPE_OK) return rc;
    t->sp_age = 0;
    t->sp_bits_age = 0;
    t->sp_shrinks = 0;
    // zone buffers: the zone, and the stale source (previous stream, n_prev - Zs <= z + last_mc symbols)
    // (>= the one-workgroup zone pass's full register window, which it loads unconditionally)
    uint64_t zneed = (gbpe_div_up((uint64_t)z + prev_mc + 1, TILE) + 2) * TILE;
    const uint64_t zmin = (uint64_t)(t->u16 ? zone_max<uint16_t>(1024) : zone_max<uint32_t>(1024)) + TILE;
    if (zneed < zmin) zneed = zmin;
    if (zneed > t->zcap) {
        for (int k = 0; k < 2; ++k) {
            hipFree(t->zbuf[k]);
            t->zbuf[k] = nullptr;
        }
        hipFree(t->wtmp);
        t->wtmp = nullptr;
        t->zcap = 0;
        if (hipMalloc(&t->zbuf[0], zneed * t->bps) != hipSuccess || hipMalloc(&t->zbuf[1], zneed * t->bps) != hipSuccess ||
            hipMalloc(&t->wtmp, zneed * t->bps) != hipSuccess)
            return gbpe_set_error(t->ctx, GBPE_E_OOM, "hipMalloc(zone) failed");
        t->zcap = zneed;
    }
    for (int k = 0; k < 2; ++k) TR_HIP(t, hipMemsetAsync(t->zbuf[k], 0, t->zcap * t->bps, s));
    if (z) {
        TR_HIP(t, hipMemcpyAsync(t->zbuf[0], cur + Zs, (uint64_t)z * t->bps, hipMemcpyDeviceToDevice, s));
        uint64_t sl = (uint64_t)z + prev_mc;
        if (Zs + sl > t->cap_syms) sl = t->cap_syms - Zs;
        if (sl > t->zcap) sl = t->zcap;
        TR_HIP(t, hipMemcpyAsync(t->zbuf[1], stale + Zs, sl * t->bps, hipMemcpyDeviceToDevice, s));
    }
    // states
    if (!t->zst) {
        TR_HIP(t, hipMalloc(&t->zst, sizeof(DevState)));
        TR_HIP(t, hipHostMalloc((void**)&t->h_zst, sizeof(DevState), hipHostMallocDefault));
    }
    memset(t->h_zst, 0, sizeof(DevState));
    t->h_zst->n = z;
    TR_HIP(t, hipMemcpyAsync(t->zst, t->h_zst, sizeof(DevState), hipMemcpyHostToDevice, s));
    t->h_st->B = Zs;
    t->h_st->Bp = Zs;
    t->h_st->body_rm = 0;
    t->h_st->sp_abort = 0;
    TR_HIP(t, hipMemcpyAsync(&t->st->B, &t->h_st->B, 4 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    // every rank checks the zone against the same length: the zone rank's target
    // until the first exchange reports the real one (single GPU: the real one)
    t->h_st->zlast = t->sharded ? (uint32_t)zt : z;
    t->h_st->is_last = z ? 1u : 0u;
    TR_HIP(t, hipMemcpyAsync(&t->st->zlast, &t->h_st->zlast, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->st->is_last, &t->h_st->is_last, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    {   // one byte counter per k_body workgroup, kept across entries (summed by gbpe_trainer_stats_get)
        const uint64_t need = gbpe_div_up(gbpe_div_up(cap, 32), SP_WPW_MIN) + 2;
        if (need > t->wg_cap) {
            uint64_t* nb = nullptr;
            TR_HIP(t, hipMalloc(&nb, need * sizeof(uint64_t)));
            TR_HIP(t, hipMemsetAsync(nb, 0, need * sizeof(uint64_t), s));
            if (t->wg_bytes) TR_HIP(t, hipMemcpyAsync(nb, t->wg_bytes, t->wg_cap * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
            TR_HIP(t, hipStreamSynchronize(s));
            hipFree(t->wg_bytes);
            t->wg_bytes = nb;
            t->wg_cap = need;
        }
    }
    // the zone rule's last count (sel_inline): the count of the merge before entry
    TR_HIP(t, hipMemcpyAsync(&t->st->mc_prev, &t->st->mc, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    // per-k_refresh-workgroup maxima the sparse merges select from (sel_inline)
    if (!t->part) TR_HIP(t, hipMalloc(&t->part, (uint64_t)(t->tb.nblk + 1) * sizeof(uint64_t)));
    if (!t->zseg && !t->sharded) {
        TR_HIP(t, hipMalloc(&t->zseg, sizeof(ZSegState)));
        TR_HIP(t, hipMemsetAsync(t->zseg, 0, sizeof(ZSegState), t->ctx->stream));
    }
    hipLaunchKernelGGL(k_refresh<S>, dim3(t->g_refresh), dim3(TPB), 0, s, t->st, 0u, 0, t->tb, (S*)nullptr,
                       (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(), t->part);
    GBPE_LAUNCH_CHECK(t->ctx);
    TR_HIP(t, hipStreamSynchronize(s));
    t->sp = true;
    t->zcur = 0;
    if (t->last_mc < nmc) t->last_mc = (uint32_t)nmc;   // the zone-shrink target's count until a merge runs
    ++t->sp_enters;
    t->sp_sectors = t->nsec;
    t->sp_zone = z;
    return GBPE_OK;
}

// Zone shrink at a step boundary: the zone keeps >= zt = sp_zt * last_mc + 64
// symbols (from a word start); its front moves into the body as new sectors and
// both zone buffers shift down by the moved length (B and Bp with them, so the
// stale buffer keeps its global coordinates).
template <typename S>
int sp_shrink(gbpe_trainer* t) {
    hipStream_t s = t->ctx->stream;
    DevState* hs = t->h_st;
    const uint32_t z = t->n - hs->B;
    const uint64_t zt = (uint64_t)t->sp_zt * t->last_mc + 64;
    if (t->sp_shrinks >= SP_SHRINKS || (uint64_t)z < zt * t->shrink_pct / 100 + 4096) return GBPE_OK;
    S* zc = (S*)t->zbuf[t->zcur];
    S* zo = (S*)t->zbuf[t->zcur ^ 1];
    hipLaunchKernelGGL(k_sp_zone_start<S>, dim3(1), dim3(1024), 0, s, (const S*)zc, (uint32_t)(z - zt), t->d_u32);
    GBPE_LAUNCH_CHECK(t->ctx);
    uint32_t L = 0;
    TR_HIP(t, hipMemcpyAsync(&L, t->d_u32, 4, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (L < 4096) return GBPE_OK;
    if (t->lex) {   // the front's words join the lexicon (deduplicated among themselves)
        LxPlan lp;
        int rc = lx_analyze<S>(t, (const S*)zc, L, false, lp);
        if (rc == GBPE_OK && lp.ok) rc = lx_commit<S>(t, lp, (const S*)zc, false);
        if (rc != GBPE_OK) return rc;
        if (!lp.ok) return GBPE_OK;   // (a collision or no room): the zone keeps its front this time
    } else {
        if ((uint64_t)t->bend + L > t->cap_syms) return GBPE_OK;
        S* body = (S*)t->buf[t->bcur];
        TR_HIP(t, hipMemcpyAsync(body + t->bend, zc, (uint64_t)L * t->bps, hipMemcpyDeviceToDevice, s));
        int rc = sp_add_sectors<S>(t, t->bend, L);
        if (rc != GBPE_OK) return rc;
    }
    const uint64_t rest = t->zcap - L;
    TR_HIP(t, hipMemcpyAsync(t->wtmp, zc + L, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemcpyAsync(zc, t->wtmp, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemcpyAsync(t->wtmp, zo + L, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemcpyAsync(zo, t->wtmp, rest * t->bps, hipMemcpyDeviceToDevice, s));
    TR_HIP(t, hipMemsetAsync(zc + rest, 0, (uint64_t)L * t->bps, s));
    TR_HIP(t, hipMemsetAsync(zo + rest, 0, (uint64_t)L * t->bps, s));
    hs->B += L;
    hs->Bp += L;
    t->h_zst->n = z - L;
    TR_HIP(t, hipMemcpyAsync(&t->st->B, &hs->B, 2 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->zst->n, &t->h_zst->n, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    ++t->sp_shrinks;
    return GBPE_OK;
}

// sparse → dense: the body sectors gathered in order into the other dense
// buffer, the zone appended; the old body buffer becomes the stale buffer, with
// the zone's stale buffer at its global place (positions >= Bp: the only ones the
// next merge's stale window can read).
template <typename S>
int sp_exit(gbpe_trainer* t) {
    hipStream_t s = t->ctx->stream;
    DevState* hs = t->h_st;
    TR_HIP(t, hipMemcpyAsync(hs, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    const uint32_t B = hs->B, Bp = hs->Bp, n = hs->n;
    const uint32_t z = n - B;
    S* body = (S*)t->buf[t->bcur];
    S* dst = (S*)t->buf[t->bcur ^ 1];
    const uint32_t nsec = t->nsec;
    uint64_t btot = 0;
    if (t->lex) {
        int rc = lx_expand<S>(t, dst, &btot);
        if (rc != GBPE_OK) return rc;
    } else {
        hipLaunchKernelGGL(k_sp_counts, dim3((uint32_t)gbpe_div_up(nsec, 256)), dim3(256), 0, s, (const uint2*)t->sec, nsec,
                           t->sp_loc);
        const uint64_t nblk = gbpe_div_up(nsec, SCAN_BLK);
        hipLaunchKernelGGL(k_chunk_scan1, dim3((uint32_t)nblk), dim3(SCAN_TPB), 0, s, (const uint32_t*)t->sp_loc,
                           (uint64_t)nsec, t->sp_loc, t->sp_blk);
        hipLaunchKernelGGL(k_chunk_scan2, dim3(1), dim3(SCAN_TPB), 0, s, t->sp_blk, nblk, t->sp_blk + nblk);
        hipLaunchKernelGGL(k_sp_gather<S>, dim3((uint32_t)gbpe_div_up(nsec, TPB / 64)), dim3(TPB), 0, s, (const S*)body,
                           (const uint2*)t->sec, nsec, (const uint32_t*)t->sp_loc, (const uint64_t*)t->sp_blk, dst);
        GBPE_LAUNCH_CHECK(t->ctx);
        TR_HIP(t, hipMemcpyAsync(&btot, t->sp_blk + nblk, 8, hipMemcpyDeviceToHost, s));
    }
    TR_HIP(t, hipMemcpyAsync(dst + B, t->zbuf[t->zcur], (uint64_t)z * t->bps, hipMemcpyDeviceToDevice, s));
    // zero the rest of the dense buffer's padding the kernels may read (halo / look-ahead)
    TR_HIP(t, hipMemsetAsync(dst + n, 0, (t->cap_syms - n) * t->bps, s));
    uint64_t sl = t->zcap;
    if (Bp + sl > t->cap_syms) sl = t->cap_syms - Bp;
    TR_HIP(t, hipMemcpyAsync(body + Bp, t->zbuf[t->zcur ^ 1], sl * t->bps, hipMemcpyDeviceToDevice, s));
    hs->sp_abort = 0;
    TR_HIP(t, hipMemcpyAsync(&t->st->sp_abort, &hs->sp_abort, 4, hipMemcpyHostToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (btot != B) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "sparse exit: body sectors hold %llu symbols, expected %u",
                                         (unsigned long long)btot, B);
    t->cur = t->bcur ^ 1;
    t->sp = false;
    t->lex = false;
    ++t->sp_exits;
    return GBPE_OK;
}

int sp_exit_any(gbpe_trainer* t) { return !t->sp ? GBPE_OK : (t->u16 ? sp_exit<uint16_t>(t) : sp_exit<uint32_t>(t)); }

}  // namespace

namespace {
// a trainer continuing from an exported state (gbpe_trainer_create_from_state):
// `bytes` is then the current u32 stream, `prev` the previous one
struct StateInit {
    const uint32_t* prev;
    uint64_t n_prev;
};

int trainer_create_impl(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                        int input_on_device, const gbpe_train_opts* opts, uint64_t cap_extra, gbpe_trainer** out,
                        const StateInit* si = nullptr) {
    if (!ctx || !out || !opts) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *out = nullptr;
    if (n == 0) return gbpe_set_error(ctx, GBPE_E_EMPTY, "No symbols to train on — corpus is empty after pre-processing");
    if (!bytes) return gbpe_set_error(ctx, GBPE_E_INVALID, "bytes is null");
    if (n >= 0xFFFFFFF0ull) return gbpe_set_error(ctx, GBPE_E_INVALID, "corpus too large for one device (%llu symbols)", (unsigned long long)n);
    auto* t = new (std::nothrow) gbpe_trainer();
    if (!t) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    t->ctx = ctx;
    t->flags = opts->flags;
    t->batch = opts->batch_size ? opts->batch_size : GBPE_BATCH_SIZE;
    const uint32_t vocab_size = opts->vocab_size ? opts->vocab_size : 256u;
    const uint32_t next_id = opts->next_token_id ? opts->next_token_id : 256u;
    t->needed = opts->target_vocab_size > vocab_size ? opts->target_vocab_size - vocab_size : 0u;
    // u16 symbols when every id the run can produce fits in 15 bits
    const uint64_t max_id = (uint64_t)next_id + t->needed;    // exclusive
    t->u16 = max_id <= 0x8000ull;
    t->max_id = (uint32_t)(max_id < 0x10000ull ? max_id : 0x10000ull);
    if (const char* e = getenv("GBPE_SPARSE_DIV")) t->sp_div = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("GBPE_REFRESH_BLOCKS")) t->refresh_blocks = (uint32_t)atoi(e);
    if (const char* e = getenv("GBPE_REHASH")) t->rehash_on = atoi(e) != 0;
    t->body_cap = (uint32_t)(ctx->num_cu > 0 ? ctx->num_cu : 256);   // one per CU: measured best at 1 GiB (128/192/256/384/512/1024: 3.01/2.42/2.14/2.66/2.45/2.98 s)
    if (const char* e = getenv("GBPE_BODY_WG")) t->body_cap = std::max<uint32_t>(1, (uint32_t)atoi(e));
    if (const char* e = getenv("GBPE_SPARSE_ZT")) t->sp_zt = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("GBPE_LEXICON")) t->lex_on = atoi(e) != 0;
    if (const char* e = getenv("GBPE_TAIL")) t->tail_on = atoi(e) != 0;
    if (const char* e = getenv("GBPE_ZONE16")) t->zone16 = atoi(e) != 0;
    if (const char* e = getenv("GBPE_TAIL_MC")) t->tail_mc = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("GBPE_LEXICON_DIV")) t->lx_div = std::max<uint32_t>(8, (uint32_t)strtoul(e, nullptr, 10));
    if (const char* e = getenv("GBPE_SUBSTEP_ZONE")) t->sub_zone = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("GBPE_SUBSTEP")) t->sub_k = std::max<uint32_t>(2, (uint32_t)strtoul(e, nullptr, 10)) & ~1u;
    if (const char* e = getenv("GBPE_DELTA_MT")) t->delta_mt = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("GBPE_DELTA_TPW")) {
        const uint32_t v = (uint32_t)strtoul(e, nullptr, 10);
        t->delta_tpw = v >= 32 ? 32 : v >= 16 ? 16 : 8;
    }
    if (const char* e = getenv("GBPE_SHRINK_PCT")) t->shrink_pct = std::max<uint32_t>(110, (uint32_t)strtoul(e, nullptr, 10));
    if (const char* e = getenv("GBPE_ZONE_SEG")) t->zseg_mode = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("GBPE_ZONE_F")) t->zone_f = std::max<uint32_t>(3, (uint32_t)strtoul(e, nullptr, 10));
    if (t->sp_zt < t->zone_f) t->sp_zt = t->zone_f;
    if (const char* e = getenv("GBPE_SPARSE_TRACE")) {
        t->trace = fopen(e, "w");
        if (t->trace && (hipMalloc(&t->d_clog, (size_t)t->batch * 8) != hipSuccess ||
                         hipHostMalloc((void**)&t->h_clog, (size_t)t->batch * 8, hipHostMallocDefault) != hipSuccess))
            t->d_clog = nullptr, t->h_clog = nullptr;   // trace without candidate counts
    }
    t->bps = t->u16 ? 2 : 4;
    t->n0 = n;
    t->n = (uint32_t)n;
    hipStream_t s = ctx->stream;
    auto fail = [&](int code) {
        gbpe_trainer_destroy(t);
        return code;
    };
    // buffers padded to whole tiles (+1 tile for the halo / next-word reads); a
    // shard may also grow by appended stale windows (cap_extra symbols)
    if (n + cap_extra >= 0xFFFFFFF0ull - 2 * TILE)
        return fail(gbpe_set_error(ctx, GBPE_E_INVALID, "shard capacity too large for one device"));
    const uint64_t ntiles0 = gbpe_div_up(n + cap_extra, TILE);
    t->cap_syms = (ntiles0 + 1) * TILE;
    for (int k = 0; k < 2; ++k) {
        if (hipMalloc(&t->buf[k], t->cap_syms * t->bps) != hipSuccess)
            return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(symbols) failed"));
        // both ping-pong buffers start zeroed, as WebGPU zero-initialises buffers
        if (hipMemsetAsync(t->buf[k], 0, t->cap_syms * t->bps, s) != hipSuccess)
            return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "memset failed"));
    }
    // pair table
    // distinct pairs start below 65536 (byte pairs) and grow by a few per merge
    // (1 GiB English at 32K: 170K live, 243K slots used): start at 2^20 slots and
    // grow when crowded (trainer_step_once).  An oversized table costs every merge:
    // k_refresh scans one dirty flag per 256-slot block (2^24 slots: 65,536 flags,
    // 1,024 workgroups) and sel_inline reduces one partial maximum per k_refresh
    // workgroup.
    uint32_t lg = opts->table_log2;
    if (lg == 0) lg = 20;
    if (lg < BLK_LOG2 + 1) lg = BLK_LOG2 + 1;
    if (lg > 28) lg = 28;
    t->table_log2 = lg;
    const uint64_t slots = 1ull << lg;
    t->tb.mask = (uint32_t)(slots - 1);
    t->tb.nblk = (uint32_t)(slots >> BLK_LOG2);
    if (hipMalloc(&t->tb.slots, slots * sizeof(uint2)) != hipSuccess ||
        hipMalloc(&t->tb.bmax, t->tb.nblk * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&t->tb.dirty, t->tb.nblk * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->tb.dlist, (t->tb.nblk + 1) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->tb.blive, t->tb.nblk * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->hitmask, (ntiles0 + 1) * TPB * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->tile_cnt, (ntiles0 + 1) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->grpsum, (ntiles0 / GRP + 2) * GSTR * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->st, sizeof(DevState)) != hipSuccess ||
        hipMalloc(&t->d_log, (size_t)t->batch * 4 * sizeof(uint32_t)) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(training buffers) failed"));
    if (hipHostMalloc((void**)&t->h_st, sizeof(DevState), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&t->h_log, (size_t)t->batch * 4 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipHostMalloc failed"));
    t->tb.used = &t->st->used;
    t->g_refresh = grid_blocks(ctx, t->tb.nblk, 2);
    if (t->refresh_blocks) t->g_refresh = std::max<uint32_t>(t->refresh_blocks, (uint32_t)gbpe_div_up(t->tb.nblk, 64));
    if (hipMemsetAsync(t->tb.dirty, 0, t->tb.nblk * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(t->hitmask, 0, (ntiles0 + 1) * TPB * sizeof(uint32_t), s) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "memset failed"));
    DevState init{};
    init.n = (uint32_t)n;
    init.next_id = next_id;
    if (si && si->n_prev > n) {   // the last merge's count (the zone rule's mc_prev)
        init.mc = (uint32_t)(si->n_prev - n);
        t->last_mc = init.mc;
        t->n_prev0 = si->n_prev;
    }
    memcpy(t->h_st, &init, sizeof(init));
    if (hipMemcpyAsync(t->st, t->h_st, sizeof(DevState), hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "state upload failed"));
    auto finish = [&]() -> int {
        if (t->flags & GBPE_TRAIN_TIMING) {
            t->evs.resize(5 * t->batch);
            for (auto& e : t->evs)
                if (hipEventCreate(&e) != hipSuccess) return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "hipEventCreate failed"));
        }
        if (hipStreamSynchronize(s) != hipSuccess) return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "trainer init failed"));
        *out = t;
        return GBPE_OK;
    };
    if (si) {   // both ping-pong buffers from u32 streams (host or device resident)
        const uint32_t* d_cur = (const uint32_t*)bytes;
        const uint32_t* d_prev = si->prev;
        void* tmp = nullptr;
        if (!input_on_device) {
            if (hipMalloc(&tmp, (n + si->n_prev) * 4 + 4) != hipSuccess)
                return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(state) failed"));
            uint32_t* h = (uint32_t*)tmp;
            if (hipMemcpyAsync(h, bytes, n * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
                (si->n_prev && hipMemcpyAsync(h + n, si->prev, si->n_prev * 4, hipMemcpyHostToDevice, s) != hipSuccess)) {
                hipFree(tmp);
                return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "state upload failed"));
            }
            d_cur = h;
            d_prev = h + n;
        }
        auto imp = [&](const uint32_t* src, void* dst, uint64_t cnt) {
            if (!cnt) return;
            const uint32_t g = (uint32_t)gbpe_div_up(cnt, TPB);
            if (t->u16)
                hipLaunchKernelGGL(k_import_symbols<uint16_t>, dim3(g), dim3(TPB), 0, s, src, (uint16_t*)dst, cnt);
            else
                hipLaunchKernelGGL(k_import_symbols<uint32_t>, dim3(g), dim3(TPB), 0, s, src, (uint32_t*)dst, cnt);
        };
        imp(d_cur, t->buf[0], n);
        if (d_prev) imp(d_prev, t->buf[1], si->n_prev);
        const bool launched = hipGetLastError() == hipSuccess;
        int rc = launched ? table_rebuild(t) : gbpe_set_error(ctx, GBPE_E_DEVICE, "symbol import launch failed");
        hipStreamSynchronize(s);
        hipFree(tmp);
        if (rc != GBPE_OK) return fail(rc);
        return finish();
    }
    // symbols: bytes (+ mask) → S with word-start bit; input may be host or device resident
    const uint8_t* d_bytes = bytes;
    const uint8_t* d_ws = word_starts;
    void* tmp = nullptr;
    if (!input_on_device) {
        const uint64_t need = n * (word_starts ? 2 : 1);
        if (hipMalloc(&tmp, need) != hipSuccess) return fail(gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(input) failed"));
        if (hipMemcpyAsync(tmp, bytes, n, hipMemcpyHostToDevice, s) != hipSuccess ||
            (word_starts && hipMemcpyAsync((uint8_t*)tmp + n, word_starts, n, hipMemcpyHostToDevice, s) != hipSuccess)) {
            hipFree(tmp);
            return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "input upload failed"));
        }
        d_bytes = (const uint8_t*)tmp;
        d_ws = word_starts ? (const uint8_t*)tmp + n : nullptr;
    }
    uint8_t* d_gpt4 = nullptr;   // GPT-4 rule word starts computed on the device (pre_tokenizer.mjs:226-292)
    if (!d_ws && (opts->flags & GBPE_TRAIN_GPT4_BOUNDARIES)) {
        int rc2 = hipMalloc(&d_gpt4, n) == hipSuccess ? gbpe_pretok_gpt4_launch(ctx, d_bytes, n, d_gpt4) : GBPE_E_OOM;
        if (rc2 != GBPE_OK) {
            if (tmp) hipFree(tmp);
            hipFree(d_gpt4);
            return fail(rc2 == GBPE_E_OOM ? gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(word starts) failed") : rc2);
        }
        d_ws = d_gpt4;
    }
    const uint32_t gb = (uint32_t)gbpe_div_up(n, TPB);
    if (t->u16)
        hipLaunchKernelGGL(k_symbols<uint16_t>, dim3(gb), dim3(TPB), 0, s, d_bytes, d_ws, (uint16_t*)t->buf[0], n,
                           (uint8_t*)nullptr);
    else
        hipLaunchKernelGGL(k_symbols<uint32_t>, dim3(gb), dim3(TPB), 0, s, d_bytes, d_ws, (uint32_t*)t->buf[0], n,
                           (uint8_t*)nullptr);
    if (hipGetLastError() != hipSuccess) {
        if (tmp) hipFree(tmp);
        return fail(gbpe_set_error(ctx, GBPE_E_DEVICE, "symbol kernel launch failed"));
    }
    int rc = table_rebuild(t);
    if (tmp || d_gpt4) {
        hipStreamSynchronize(s);
        hipFree(tmp);
        hipFree(d_gpt4);
    }
    if (rc != GBPE_OK) return fail(rc);
    return finish();
}
}  // namespace

extern "C" int gbpe_trainer_create(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                                   int input_on_device, const gbpe_train_opts* opts, gbpe_trainer** out) {
    return trainer_create_impl(ctx, bytes, n, word_starts, input_on_device, opts, 0, out);
}

extern "C" int gbpe_trainer_create_from_state(gbpe_ctx* ctx, const uint32_t* cur, uint64_t n, const uint32_t* prev,
                                              uint64_t n_prev, int input_on_device, const gbpe_train_opts* opts,
                                              gbpe_trainer** out) {
    if (n_prev < n) return gbpe_set_error(ctx, GBPE_E_INVALID, "create_from_state: n_prev (%llu) < n (%llu)",
                                          (unsigned long long)n_prev, (unsigned long long)n);
    if (n_prev > n && !prev) return gbpe_set_error(ctx, GBPE_E_INVALID, "create_from_state: prev is null");
    const StateInit si{prev, n_prev};
    return trainer_create_impl(ctx, (const uint8_t*)cur, n, nullptr, input_on_device, opts, n_prev - n, out, &si);
}

namespace {
int trainer_step_once(gbpe_trainer* t, uint32_t max_merges, uint32_t* merges_out, uint32_t* n_done, uint32_t* early_stop) {
    if (n_done) *n_done = 0;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    uint32_t k = max_merges ? max_merges : t->batch;
    if (k > t->batch) k = t->batch;
    if (t->done + k > t->needed) k = t->needed - t->done;
    if (t->stop || k == 0) return GBPE_OK;
    hipStream_t s = t->ctx->stream;
    // rebuild the pair table when it gets crowded (dead pairs accumulate), twice as
    // large (or more) while the live pairs would fill over a quarter of it
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    if ((uint64_t)t->h_st->used * 2 > slots) {
        const uint64_t live = std::max<uint64_t>(t->h_st->live, t->h_st->used / 2);
        uint32_t lg = t->table_log2;
        while (lg < 28 && live * 4 > (1ull << lg)) ++lg;
        int rc;
        if (t->sp && !t->sharded && t->rehash_on) {   // the sparse loop goes on over the moved entries
            rc = table_rehash(t, lg);
        } else {
            rc = sp_exit_any(t);   // the full recount runs on the dense stream
            if (rc == GBPE_OK && lg != t->table_log2) rc = table_resize(t, lg);
            if (rc == GBPE_OK) rc = table_rebuild(t);
        }
        if (rc != GBPE_OK) return rc;
        ++t->table_grows;
    }
    // sector-sparse loop once merges touch a small fraction of the stream
    if (t->sp_cooldown) {
        --t->sp_cooldown;
    } else if (!t->sp && !t->sharded && !(t->flags & GBPE_TRAIN_DENSE_ONLY)) {
        // with the word lexicon the body costs what its distinct words cost, so the
        // loop can enter as soon as the zone (~7 x the next count) is a small part of
        // the stream — before the first merge; without it, once counts
        // are a 1/sp_div fraction
        // with the lexicon the decision (and the zone) follow the NEXT merge's count,
        // the table maximum: one huge first merge (C5's (32,32), 17 % of the stream)
        // then ends only a one-merge dense step (enter_lim below)
        uint32_t mc = t->last_mc, next = 0;
        if (t->lex_on) {
            if (!t->d_u32) TR_HIP(t, hipMalloc(&t->d_u32, 64));
            hipLaunchKernelGGL(k_topcount, dim3(1), dim3(1024), 0, s, t->tb, t->d_u32);
            GBPE_LAUNCH_CHECK(t->ctx);
            TR_HIP(t, hipMemcpyAsync(&next, t->d_u32, 4, hipMemcpyDeviceToHost, s));
            TR_HIP(t, hipStreamSynchronize(s));
            mc = next;
        }
        const uint64_t div = t->lex_on ? t->lx_div : t->sp_div;
        const bool count_ok = mc && ((t->flags & GBPE_TRAIN_SPARSE_EARLY) || (uint64_t)mc * div <= t->n);
        if (count_ok) {
            int rc = t->u16 ? sp_enter<uint16_t>(t, true, next) : sp_enter<uint32_t>(t, true, next);
            if (rc != GBPE_OK) return rc;
        }
        // still dense with the lexicon on: the device ends the step once a merge's count
        // would pass the entry test, so the loop enters at the next step boundary
        const uint32_t lim = (!t->sp && t->lex_on && mc && !count_ok) ? (uint32_t)(t->n / div) : 0u;
        if (lim != t->h_st->enter_lim) {
            t->h_st->enter_lim = lim;
            TR_HIP(t, hipMemcpyAsync(&t->st->enter_lim, &t->h_st->enter_lim, sizeof(uint32_t), hipMemcpyHostToDevice, s));
        }
    }
    // keep the zone near its minimum, then rebuild stale filters now and then
    if (t->sp) {
        int rc = t->u16 ? sp_shrink<uint16_t>(t) : sp_shrink<uint32_t>(t);
        if (rc != GBPE_OK) return rc;
    }
    if (t->sp && t->sp_age >= 4096) {   // signatures saturate faster than the token bitmap goes stale
        const bool wb = t->sp_bits_age >= 16384;
        int rc = t->u16 ? sp_filters<uint16_t>(t, wb) : sp_filters<uint32_t>(t, wb);
        if (rc != GBPE_OK) return rc;
    }
    // waiting for the lexicon entry on a long stream: one merge per step (a dense merge
    // costs milliseconds there; every round the step enqueues after the entry point
    // would still launch its full-grid kernels as no-ops)
    if (!t->sp && t->h_st->enter_lim && t->n >= (1u << 24)) k = 1;
    // a large zone shrinks every sub_k merges instead of every step (early counts fall fast)
    if (t->sp && t->n - t->h_st->B > t->sub_zone && k > t->sub_k) k = t->sub_k;
    // reset the per-step counter + budget (trainer.js:239)
    DevState* hs = t->h_st;
    hs->merges_done = 0;
    hs->budget = k;
    TR_HIP(t, hipMemcpyAsync(&t->st->merges_done, &hs->merges_done, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->st->budget, &hs->budget, sizeof(uint32_t), hipMemcpyHostToDevice, s));
#ifdef GBPE_KTRACE
    if (getenv("GBPE_KTRACE_OUT")) {
        static unsigned long long* kbuf = nullptr;
        if (!kbuf) {
            const size_t nb = (size_t)(KT_MERGES / KT_EVERY) * 2 * KT_WG * KT_SLOTS * 8;
            TR_HIP(t, hipMalloc(&kbuf, nb));
            TR_HIP(t, hipMemsetAsync(kbuf, 0, nb, s));
            TR_HIP(t, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ktr), &kbuf, sizeof(kbuf), 0, hipMemcpyHostToDevice, s));
        }
        const uint32_t kb = (uint32_t)t->done;
        TR_HIP(t, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_kt_base), &kb, 4, 0, hipMemcpyHostToDevice, s));
    }
#endif
    if (t->sp) {
        hs->sel_round = 0;
        TR_HIP(t, hipMemcpyAsync(&t->zst->merges_done, &hs->merges_done, sizeof(uint32_t), hipMemcpyHostToDevice, s));
        TR_HIP(t, hipMemcpyAsync(&t->st->sel_round, &hs->sel_round, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    }
    const uint64_t ntiles = gbpe_div_up(t->n, TILE);
    // tile blocks + stale-tail blocks (the window is at most mc <= n/2 symbols)
    const uint32_t g_tail = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u
                            : grid_persistent(t->ctx, gbpe_div_up(t->n / 2 + 1, TPB * 16), 1);
    const uint32_t g_delta = (uint32_t)(ntiles ? ntiles : 1);
    const uint32_t g_compact = (uint32_t)ntiles + g_tail;
    const uint32_t g_refresh = t->g_refresh;
    const bool timing = (t->flags & GBPE_TRAIN_TIMING) != 0;
    const bool sparse = t->sp;
    SpGrid sg{};
    if (sparse) {
        const uint32_t zn = t->n - hs->B;   // zone length (it only shrinks within a step)
        const uint64_t zt = gbpe_div_up(zn, TILE);
        const uint32_t z256 = t->u16 ? zone_max<uint16_t>(256) : zone_max<uint32_t>(256);
        sg.bt = zn <= z256 ? 256 : 1024;   // small zone: the low-latency 256-thread workgroups
        body_grid(t, sg.bt, &sg.body, &sg.wpg);
        if (sg.bt == 1024 && t->u16 && zn <= 16384u && t->zone16) sg.bt = 1023;
        sg.zone1 = zn <= (t->u16 ? zone_max<uint16_t>(sg.bt) : zone_max<uint32_t>(sg.bt)) ? 1u : 0u;
        // a zone of 16K-1M symbols: 16K-symbol segments inside k_body (its ZSEG form)
        const uint32_t zs_lo = t->zseg_mode == 2 ? (t->u16 ? zone_max<uint16_t>(1024) : zone_max<uint32_t>(1024)) : 16384u;
        if (t->zseg_mode && t->zseg && zn > zs_lo && zn <= NSEG_MAX * 16384u)
            sg.zone1 = (uint32_t)gbpe_div_up(zn, 16384u);
        sg.copy = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u : grid_persistent(t->ctx, gbpe_div_up(zn / 5 + 1, TPB * 8), 1);
        sg.zdelta = (uint32_t)(zt ? zt : 1);
        sg.ztail = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u
                                                           : (uint32_t)std::min<uint64_t>(1024, gbpe_div_up(zn / 5 + 1, 2048));
        sg.zcompact = (uint32_t)zt + ((t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 0u
                                      : grid_persistent(t->ctx, gbpe_div_up(zn / 2 + 1, TPB * 16), 1));
        sg.refresh = g_refresh;
    }
    // the persistent tail loop: one workgroup, the whole step
#ifdef GBPE_TAIL_LOOP
    const uint32_t zn_now = sparse ? t->n - hs->B : 0u;
    const bool tail = sparse && t->tail_on && !t->tail_skip && !t->sharded && t->last_mc <= t->tail_mc &&
                      zn_now <= (t->u16 ? zone_max<uint16_t>(TL_BT) : zone_max<uint32_t>(TL_BT)) &&
                      t->tb.nblk <= (TL_MAXG << TL_GRP);
    t->tail_skip = false;
    auto launch_tail = [&]() -> int {
        if (!t->d_tstat) TR_HIP(t, hipMalloc(&t->d_tstat, 16));
        if (timing) TR_HIP(t, hipEventRecord(t->evs[0], s));
        const uint32_t wused = (uint32_t)gbpe_div_up(t->nsec, 32);
        const bool ex = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) != 0;
#define GBPE_TAIL_LAUNCH(S_, E_)                                                                                     \
        do {                                                                                                         \
        if (zn_now <= (uint32_t)TL_BT * 8u)                                                                         \
            hipLaunchKernelGGL((k_tail<S_, E_, 8>), dim3(1), dim3(TL_BT), 0, s, t->st, t->zst, (S_*)sp_body(t), sp_mul(t), \
                               t->sec, t->bits, t->W, wused, t->sig, t->tb, (S_*)t->zbuf[t->zcur],                      \
                               (S_*)t->zbuf[t->zcur ^ 1], t->d_log, t->wg_bytes, t->d_tstat);                          \
        else                                                                                                         \
        hipLaunchKernelGGL((k_tail<S_, E_, ZoneDim<S_, TL_BT>::ZPT>), dim3(1), dim3(TL_BT), 0, s, t->st, t->zst, (S_*)sp_body(t), sp_mul(t), t->sec, \
                           t->bits, t->W, wused, t->sig, t->tb, (S_*)t->zbuf[t->zcur], (S_*)t->zbuf[t->zcur ^ 1], t->d_log,   \
                           t->wg_bytes, t->d_tstat);                                                             \
        hipLaunchKernelGGL(k_refresh<S_>, dim3(t->g_refresh), dim3(TPB), 0, s, t->st, 0u, 0, t->tb, (S_*)nullptr,    \
                           (const uint32_t*)nullptr, (DevState*)nullptr, (uint32_t*)nullptr, FusedSel(), t->part); \
        } while (0)
        if (t->u16) {
            if (ex) GBPE_TAIL_LAUNCH(uint16_t, true);
            else GBPE_TAIL_LAUNCH(uint16_t, false);
        } else {
            if (ex) GBPE_TAIL_LAUNCH(uint32_t, true);
            else GBPE_TAIL_LAUNCH(uint32_t, false);
        }
#undef GBPE_TAIL_LAUNCH
        GBPE_LAUNCH_CHECK(t->ctx);
        if (timing) TR_HIP(t, hipEventRecord(t->evs[1], s));
        return GBPE_OK;
    };
#else
    const bool tail = false;   // (diagnostic build only: -DGBPE_TAIL_LOOP, tools/build_variant.sh)
    auto launch_tail = [&]() -> int { return GBPE_OK; };
#endif
    auto launch_all = [&]() -> int {
        if (tail) return launch_tail();
        for (uint32_t r = 0; r < k; ++r) {
            hipEvent_t* ev = timing ? &t->evs[5 * r] : nullptr;
            int rc;
            if (sparse)
                rc = t->u16 ? launch_merge_sparse<uint16_t>(t, r, s, sg, timing, ev)
                            : launch_merge_sparse<uint32_t>(t, r, s, sg, timing, ev);
            else
                rc = t->u16 ? launch_merge<uint16_t>(t, r, s, g_delta, g_compact, g_refresh, timing, ev)
                            : launch_merge<uint32_t>(t, r, s, g_delta, g_compact, g_refresh, timing, ev);
            if (rc != GBPE_OK) return rc;
        }
        return GBPE_OK;
    };
    {
        int rc = launch_all();
        if (rc != GBPE_OK) return rc;
        if (sparse) hipLaunchKernelGGL(k_live, dim3(1), dim3(1024), 0, s, t->st, t->tb);
    }
    TR_HIP(t, hipMemcpyAsync(t->h_st, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipMemcpyAsync(t->h_log, t->d_log, (size_t)k * 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (sparse) TR_HIP(t, hipMemcpyAsync(t->h_zst, t->zst, sizeof(DevState), hipMemcpyDeviceToHost, s));
    if (sparse && t->d_clog) TR_HIP(t, hipMemcpyAsync(t->h_clog, t->d_clog, (size_t)k * 8, hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    const uint32_t done = hs->merges_done;
    const uint32_t err = hs->err | (sparse ? t->h_zst->err : 0u);
    if (err) {
        return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "training invariant violated (err=0x%x: %s%s%s%s%s)", err,
                              (err & ERR_TABLE_FULL) ? "pair table full " : "",
                              (err & ERR_COUNT_MISMATCH) ? "survivor count mismatch " : "",
                              (err & ERR_PAIR_MISSING) ? "selected pair missing " : "",
                              (err & ERR_SPARSE_WINDOW) ? "sparse stale window outside the zone " : "",
                              (err & ERR_SPIN) ? "zone segment hand-off timed out" : "");
    }
    if (timing && tail) {
        float ms = 0;
        hipEventElapsedTime(&ms, t->evs[0], t->evs[1]);
        t->ms_tail += ms;
        t->ms_sparse += ms;
        t->timed_merges += done;
    } else if (timing) {
        for (uint32_t r = 0; r < done; ++r) {
            float a = 0, b = 0, c = 0, d1 = 0, d2 = 0;
            hipEvent_t* ev = &t->evs[5 * r];
            hipEventElapsedTime(&a, ev[0], ev[1]);
            hipEventElapsedTime(&b, ev[1], ev[2]);
            hipEventElapsedTime(&c, ev[2], ev[4]);
            hipEventElapsedTime(&d1, ev[1], ev[3]);
            hipEventElapsedTime(&d2, ev[3], ev[2]);
            t->ms_select += a;
            t->ms_merge += b;
            t->ms_other += c;
            t->ms_delta += d1;
            t->ms_compact += d2;
            (sparse ? t->ms_sparse : t->ms_dense) += b;
            if (sparse) t->ms_body += d1;
        }
        t->timed_merges += done;
    }
    // algorithmic stream bytes: s * (2 N_i + N_{i+1})
    uint64_t N = t->n;
    for (uint32_t r = 0; r < done; ++r) {
        const uint64_t mc = t->h_log[r * 4 + 3];
        t->bytes_moved += (uint64_t)t->bps * (2 * N + (N - mc));
        if (!sparse) t->dense_bytes += (uint64_t)t->bps * (2 * N + (N - mc));
        N -= mc;
        if (merges_out) memcpy(merges_out + 4 * r, t->h_log + 4 * r, 4 * sizeof(uint32_t));
    }
    t->n = hs->n;
    if (N != t->n) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "host/device symbol count disagree");
    if (done) t->last_mc = t->h_log[(done - 1) * 4 + 3];
    if (t->trace) {   // merge index, count, stream length before, sparse, candidate sectors, sectors with sites
        uint64_t nn = N;
        for (uint32_t r = done; r-- > 0;) nn += t->h_log[r * 4 + 3];
        for (uint32_t r = 0; r < done; ++r) {
            fprintf(t->trace, "%u %u %llu %d %u %u\n", t->done + r, t->h_log[r * 4 + 3], (unsigned long long)nn,
                    sparse ? 1 : 0, sparse && t->h_clog ? t->h_clog[2 * r] : 0u, sparse && t->h_clog ? t->h_clog[2 * r + 1] : 0u);
            nn -= t->h_log[r * 4 + 3];
        }
    }
    if (tail) {
        t->tail_merges += done;
        ++t->tail_steps;
        if (done < k && !hs->stop && !hs->sp_abort) {   // left early (LDS lists): k_body finishes the step
            t->tail_skip = true;
            ++t->tail_exits;
            if (done == 0) {   // (its first merge did not fit): run the step with k_body now
                return trainer_step_once(t, max_merges, merges_out, n_done, early_stop);
            }
        }
    }
    if (sparse) {
        t->zcur ^= (int)(done & 1u);
        t->sp_merges += done;
        t->sp_age += done;
        t->sp_bits_age += done;
        if (hs->sp_abort) {   // a merge outgrew the zone: it was not run; continue dense
            int rc = sp_exit_any(t);
            if (rc != GBPE_OK) return rc;
            t->sp_cooldown = 1;
            if (done == 0 && !hs->stop) return trainer_step_once(t, max_merges, merges_out, n_done, early_stop);
        }
    } else {
        t->cur ^= (done & 1u);
    }
    t->done += done;
    t->stop = hs->stop != 0;
    if (n_done) *n_done = done;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    return GBPE_OK;
}
}  // namespace

// One host step of up to max_merges merges (trainer.js:225-335's 128-merge batch).
// Internally a sparse step whose zone is still large runs as several sub-steps
// (trainer_step_once), so the zone can shrink between them.
extern "C" int gbpe_trainer_step(gbpe_trainer* t, uint32_t max_merges, uint32_t* merges_out, uint32_t* n_done,
                                 uint32_t* early_stop) {
    if (!t) return GBPE_E_INVALID;
    uint32_t want = max_merges ? max_merges : t->batch;
    if (want > t->batch) want = t->batch;
    uint32_t got = 0, es = 0;
    int rc = GBPE_OK;
    while (got < want) {
        uint32_t nd = 0;
        rc = trainer_step_once(t, want - got, merges_out ? merges_out + 4 * got : nullptr, &nd, &es);
        if (rc != GBPE_OK) break;
        got += nd;
        if (nd == 0 || es) break;
    }
    if (n_done) *n_done = got;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    return rc;
}

extern "C" int gbpe_trainer_stats_get(gbpe_trainer* t, gbpe_trainer_stats* o) {
    if (!t || !o) return GBPE_E_INVALID;
    memset(o, 0, sizeof(*o));
    o->symbol_count = t->n;
    o->merges_done = t->done;
    o->stream_bytes_moved = t->bytes_moved;
    o->tail_dropped = t->h_st->tail_total;
    o->table_slots = (uint64_t)t->tb.mask + 1;
    o->table_used = t->h_st->used;
    o->bytes_per_symbol = t->bps;
    o->early_stop = t->stop;
    o->ms_merge = t->ms_merge;
    o->ms_delta = t->ms_delta;
    o->ms_compact = t->ms_compact;
    o->ms_select = t->ms_select;
    o->ms_other = t->ms_other;
    o->timed_merges = t->timed_merges;
    o->live_pairs = t->h_st->live;
    o->max_live_pairs = t->h_st->max_live;
    o->sparse_merges = t->sp_merges;
    o->sparse_enters = t->sp_enters;
    o->sparse_exits = t->sp_exits;
    o->sparse_sectors = t->sp_sectors;
    o->sparse_zone = t->sp_zone;
    o->dense_bytes = t->dense_bytes;
    o->ms_dense = t->ms_dense;
    o->ms_sparse = t->ms_sparse;
    o->ms_body = t->ms_body;
    o->zone_bytes = t->h_st->sp_bytes;
    o->lexicon_builds = (uint32_t)t->lx_builds;
    o->lexicon_fallbacks = (uint32_t)t->lx_fallbacks;
    o->lexicon_words = t->lx_words;
    o->lexicon_entries = t->lx_nuid;
    o->lexicon_symbols = t->lx_len;
    o->tail_merges = t->tail_merges;
    o->tail_steps = t->tail_steps;
    o->tail_exits = t->tail_exits;
    o->ms_tail = t->ms_tail;
    if (t->wg_bytes && t->wg_cap) {   // the per-workgroup counters of k_body (and its zone workgroup)
        std::vector<uint64_t> h(t->wg_cap);
        if (hipMemcpy(h.data(), t->wg_bytes, t->wg_cap * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess)
            for (uint64_t v : h) o->body_bytes += v;
    }
    return GBPE_OK;
}

extern "C" int gbpe_trainer_symbols(gbpe_trainer* t, uint32_t* out, uint64_t cap, uint64_t* n) {
    if (!t || !n) return GBPE_E_INVALID;
    *n = t->n;
    if (!out) return GBPE_OK;
    if (cap < t->n) return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "symbols: need %u", t->n);
    {
        int rc = sp_exit_any(t);   // back to one dense stream (training may go on; it re-enters later)
        if (rc != GBPE_OK) return rc;
    }
    hipStream_t s = t->ctx->stream;
    uint32_t* d = nullptr;
    TR_HIP(t, hipMalloc(&d, (uint64_t)t->n * 4 + 4));
    const uint32_t g = (uint32_t)gbpe_div_up(t->n, 256);
    if (t->n) {
        if (t->u16)
            hipLaunchKernelGGL(k_export_symbols<uint16_t>, dim3(g), dim3(256), 0, s, (const uint16_t*)t->buf[t->cur], d,
                               (uint64_t)t->n);
        else
            hipLaunchKernelGGL(k_export_symbols<uint32_t>, dim3(g), dim3(256), 0, s, (const uint32_t*)t->buf[t->cur], d,
                               (uint64_t)t->n);
    }
    hipError_t e = hipMemcpyAsync(out, d, (uint64_t)t->n * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(d);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "symbol export failed: %s", hipGetErrorString(e));
    return GBPE_OK;
}

// current + previous stream (consolidation).  The previous stream
// is the other ping-pong buffer over the previous length: a shard's pln, or
// n + last count on one device (zeros before the first merge).
extern "C" int gbpe_trainer_export_state(gbpe_trainer* t, uint32_t* cur, uint64_t cap_cur, uint64_t* n_cur,
                                         uint32_t* prev, uint64_t cap_prev, uint64_t* n_prev, int on_device) {
    if (!t || !n_cur || !n_prev) return GBPE_E_INVALID;
    {
        int rc = sp_exit_any(t);   // one dense stream (+ its stale buffer where the next window can read)
        if (rc != GBPE_OK) return rc;
    }
    hipStream_t s = t->ctx->stream;
    TR_HIP(t, hipMemcpyAsync(t->h_st, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    const uint64_t n = t->n;
    // (a trainer created from a state and not stepped since re-exports the imported length)
    uint64_t np = t->sharded ? (uint64_t)t->h_st->pln : (t->done ? n + t->last_mc : (t->n_prev0 ? t->n_prev0 : n));
    if (np > t->cap_syms) np = t->cap_syms;
    *n_cur = n;
    *n_prev = np;
    if (!cur && !prev) return GBPE_OK;
    if ((cur && cap_cur < n) || (prev && cap_prev < np))
        return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "export_state: need %llu + %llu", (unsigned long long)n,
                              (unsigned long long)np);
    uint32_t* d = nullptr;
    if (!on_device) TR_HIP(t, hipMalloc(&d, (n + np) * 4 + 4));
    auto exp = [&](const void* src, uint32_t* dst, uint64_t cnt) {
        if (!cnt || !dst) return;
        const uint32_t g = (uint32_t)gbpe_div_up(cnt, 256);
        if (t->u16)
            hipLaunchKernelGGL(k_export_symbols<uint16_t>, dim3(g), dim3(256), 0, s, (const uint16_t*)src, dst, cnt);
        else
            hipLaunchKernelGGL(k_export_symbols<uint32_t>, dim3(g), dim3(256), 0, s, (const uint32_t*)src, dst, cnt);
    };
    exp(t->buf[t->cur], on_device ? cur : d, n);
    exp(t->buf[t->cur ^ 1], on_device ? prev : d + n, np);
    hipError_t e = hipGetLastError();
    if (!on_device) {
        if (e == hipSuccess && cur && n) e = hipMemcpyAsync(cur, d, n * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && prev && np) e = hipMemcpyAsync(prev, d + n, np * 4, hipMemcpyDeviceToHost, s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(d);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "state export failed: %s", hipGetErrorString(e));
    return GBPE_OK;
}

extern "C" int gbpe_trainer_pair_counts(gbpe_trainer* t, uint32_t* pids, uint32_t* counts, uint64_t cap, uint64_t* n) {
    if (!t || !n) return GBPE_E_INVALID;
    hipStream_t s = t->ctx->stream;
    uint32_t* d = nullptr;
    const uint64_t c = cap ? cap : 1;
    TR_HIP(t, hipMalloc(&d, (2 * c + 1) * sizeof(uint32_t)));
    hipError_t e = hipMemsetAsync(d, 0, sizeof(uint32_t), s);
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    hipLaunchKernelGGL(k_dump_pairs, dim3((uint32_t)gbpe_div_up(slots, 256)), dim3(256), 0, s, t->tb, d + 1, d + 1 + c,
                       d, (uint32_t)cap);
    uint32_t cnt = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&cnt, d, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess && cnt <= cap && cap) {
        e = hipMemcpy(pids, d + 1, (uint64_t)cnt * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(counts, d + 1 + c, (uint64_t)cnt * 4, hipMemcpyDeviceToHost);
    }
    hipFree(d);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "pair dump failed: %s", hipGetErrorString(e));
    *n = cnt;
    if (cnt > cap) return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "pair dump: need %u", cnt);
    return GBPE_OK;
}

extern "C" void gbpe_trainer_destroy(gbpe_trainer* t) {
    if (!t) return;
    if (t->ctx && t->ctx->stream) hipStreamSynchronize(t->ctx->stream);
#ifdef GBPE_KTRACE
    if (const char* path = getenv("GBPE_KTRACE_OUT")) {   // one file per trainer: path.<done merges>
        std::vector<unsigned long long> h((size_t)(KT_MERGES / KT_EVERY) * 2 * KT_WG * KT_SLOTS);
        unsigned long long* kbuf = nullptr;
        if (hipMemcpyFromSymbol(&kbuf, HIP_SYMBOL(g_ktr), sizeof(kbuf), 0, hipMemcpyDeviceToHost) == hipSuccess && kbuf &&
            hipMemcpy(h.data(), kbuf, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            char fn[512];
            snprintf(fn, sizeof(fn), "%s.%llu", path, (unsigned long long)t->done);
            if (FILE* f = fopen(fn, "wb")) {
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
        if (kbuf) hipMemset(kbuf, 0, h.size() * 8);
    }
#endif
    for (auto& e : t->evs)
        if (e) hipEventDestroy(e);
    hipFree(t->buf[0]);
    hipFree(t->buf[1]);
    hipFree(t->tb.slots);
    hipFree(t->tb.bmax);
    hipFree(t->tb.dirty);
    hipFree(t->tb.dlist);
    hipFree(t->tb.blive);
    hipFree(t->hitmask);
    hipFree(t->tile_cnt);
    hipFree(t->grpsum);
    hipFree(t->sec);
    hipFree(t->sp_loc);
    hipFree(t->sp_blk);
    hipFree(t->bits);
    hipFree(t->sig);
    hipFree(t->zbuf[0]);
    hipFree(t->zbuf[1]);
    hipFree(t->wtmp);
    hipFree(t->zst);
    hipFree(t->d_u32);
    hipFree(t->part);
    hipFree(t->zseg);
    hipFree(t->wg_bytes);
    hipFree(t->lx_store);
    hipFree(t->lx_mul);
    hipFree(t->lx_occ);
    hipFree(t->lx_w0);
    hipFree(t->lx_tmp);
    hipFree(t->d_tstat);
    if (t->h_zst) hipHostFree(t->h_zst);
    hipFree(t->d_clog);
    if (t->h_clog) hipHostFree(t->h_clog);
    if (t->trace) fclose(t->trace);
    hipFree(t->dt.slots);
    hipFree(t->dt.dirty);
    hipFree(t->d_nlog);
    hipFree(t->rec_send);
    hipFree(t->rec_recv);
    if (t->h_nlog) hipHostFree(t->h_nlog);
    hipFree(t->st);
    hipFree(t->d_log);
    if (t->h_st) hipHostFree(t->h_st);
    if (t->h_log) hipHostFree(t->h_log);
    delete t;
}

extern "C" int gbpe_train(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                          const gbpe_train_opts* opts, gbpe_progress_cb cb, void* user, uint32_t* merges_out,
                          uint32_t merges_cap, uint32_t* n_merges, uint32_t* early_stop) {
    if (n_merges) *n_merges = 0;
    if (early_stop) *early_stop = 0;
    gbpe_trainer* t = nullptr;
    int rc = gbpe_trainer_create(ctx, bytes, n, word_starts, 0, opts, &t);
    if (rc != GBPE_OK) return rc;
    std::vector<uint32_t> batch((size_t)t->batch * 4);
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t total = 0;
    bool stopped = false;
    while (total < t->needed && !stopped) {
        uint32_t done = 0, es = 0;
        rc = gbpe_trainer_step(t, t->batch, batch.data(), &done, &es);
        if (rc != GBPE_OK) break;
        for (uint32_t i = 0; i < done; ++i) {
            if (merges_out && total + i < merges_cap) memcpy(merges_out + 4 * (total + i), &batch[4 * i], 16);
        }
        total += done;
        stopped = es != 0;
        if (cb) {
            gbpe_progress p{};
            p.merge_index = total;
            p.total_merges = t->needed;
            p.best_count = done ? batch[4 * (done - 1) + 3] : 0u;
            p.symbol_count = t->n;
            p.batch_merges = done;
            p.early_stop = stopped;
            p.elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (cb(&p, batch.data(), user) != 0) {
                rc = gbpe_set_error(ctx, GBPE_E_CANCELLED, "training cancelled by progress callback");
                break;
            }
        }
        if (done == 0 && !stopped) break;
    }
    if (n_merges) *n_merges = total < merges_cap || !merges_out ? total : merges_cap;
    if (early_stop) *early_stop = stopped ? 1u : 0u;
    if (rc == GBPE_OK && merges_out && total > merges_cap)
        rc = gbpe_set_error(ctx, GBPE_E_CAPACITY, "merges_out too small: need %u", total);
    gbpe_trainer_destroy(t);
    return rc;
}

extern "C" int gbpe_word_boundary(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, uint8_t* ws_out) {
    if (!ctx || (!bytes && n) || (!ws_out && n)) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    if (n == 0) return GBPE_OK;
    hipStream_t s = ctx->stream;
    uint8_t* d = nullptr;
    GBPE_HIP(ctx, hipMalloc(&d, 2 * n));
    hipError_t e = hipMemcpyAsync(d, bytes, n, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_symbols<uint32_t>, dim3((uint32_t)gbpe_div_up(n, TPB)), dim3(TPB), 0, s, d,
                       (const uint8_t*)nullptr, (uint32_t*)nullptr, n, d + n);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(ws_out, d + n, n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(d);
    if (e != hipSuccess) return gbpe_set_error(ctx, GBPE_E_DEVICE, "word boundary failed: %s", hipGetErrorString(e));
    return GBPE_OK;
}

// ═══ sharded training (gbpe_shard_*) ═════════════════════════════════════════
//
// One rank per GPU; every rank keeps a replica of the GLOBAL pair-count table.
// Per merge (protocol: gpubpe/sharded.py, pinned on CPU by tests/test_sharded.py):
//   phase 1  k_select (on the replica) → k_delta (local sites; deltas into the
//            per-merge delta table) → k_shard_send (delta table → record list,
//            clearing it; the header; this rank's piece of the stale-window
//            superset [gnew - mc, gnew) of the previous input stream)
//   exchange one all-gather of the fixed-size records (host loop or
//            gbpe_shard_step_comm's ncclAllGather)
//   phase 2  k_shard_recv (every rank's deltas + the window's pairs into the
//            replica, new global layout; the owner rank appends the window) →
//            k_compact (local keep limit) → k_refresh.
// A record that does not fit stalls the merge on every rank (selection undone).

namespace {


template <typename S>
__device__ __forceinline__ uint32_t to_canon(uint32_t x) {
    return (x & Sym<S>::TM) | ((x & Sym<S>::WS) ? 0x10000u : 0u);
}
template <typename S>
__device__ __forceinline__ uint32_t from_canon(uint32_t x) {
    return (x & 0xFFFFu) | ((x & 0x10000u) ? Sym<S>::WS : 0u);
}

// list role of the send kernels: the per-merge delta table's dirty blocks become
// the record's {pid, delta} list (clearing what they read); each block adds its
// entries to rec[H_L]
__device__ void shard_list_role(DevState* st, Table dt, uint32_t* __restrict__ rec, uint32_t cap_list, uint32_t nlb) {
    __shared__ uint64_t s_dmask;
    __shared__ uint32_t wcnt[TPB / 64], s_base;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t per = (dt.nblk + nlb - 1) / nlb;
    const uint32_t b0 = blockIdx.x * per;
    if (threadIdx.x < 64) {
        const uint32_t blk = b0 + threadIdx.x;
        const bool d = threadIdx.x < per && blk < dt.nblk && dt.dirty[blk];
        const unsigned long long m = __ballot(d);
        if (threadIdx.x == 0) s_dmask = m;
    }
    __syncthreads();
    uint64_t dm = s_dmask;
    constexpr int NV = (1 << BLK_LOG2) / 2 >= TPB ? (1 << BLK_LOG2) / 2 / TPB : 1;
    constexpr uint32_t NQ = (1u << BLK_LOG2) / 2;   // 16-byte quads per block
    while (dm) {
        const uint32_t blk = b0 + (uint32_t)(__ffsll((long long)dm) - 1);
        dm &= dm - 1;
        uint4* sl = reinterpret_cast<uint4*>(dt.slots + ((uint64_t)blk << BLK_LOG2));
        uint4 e[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k)
            e[k] = threadIdx.x + k * TPB < NQ ? sl[threadIdx.x + k * TPB] : make_uint4(0u, 0u, 0u, 0u);
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < NV; ++k) c += (e[k].x && e[k].y) + (e[k].z && e[k].w);
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wcnt[wid] = incl;
        __syncthreads();
        uint32_t pre = incl - c, tot = 0;
        for (int w = 0; w < TPB / 64; ++w) {
            pre += w < wid ? wcnt[w] : 0u;
            tot += wcnt[w];
        }
        if (threadIdx.x == 0) {
            s_base = tot ? atomicAdd(&st->dcount, tot) : 0u;
            if (tot) atomicAdd(&rec[H_L], tot);
            dt.dirty[blk] = 0u;
        }
        __syncthreads();
        uint32_t o = s_base + pre;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            if (e[k].x && e[k].y) {
                if (o < cap_list) { rec[HDR + 2 * o] = e[k].x; rec[HDR + 2 * o + 1] = e[k].y; }
                ++o;
            }
            if (e[k].z && e[k].w) {
                if (o < cap_list) { rec[HDR + 2 * o] = e[k].z; rec[HDR + 2 * o + 1] = e[k].w; }
                ++o;
            }
            if ((e[k].x || e[k].z) && threadIdx.x + k * TPB < NQ) sl[threadIdx.x + k * TPB] = make_uint4(0u, 0u, 0u, 0u);
        }
        __syncthreads();
    }
}

// Phase-1 send kernel, three block roles:
//   [0, nlb)        delta table (dirty blocks only) → record list {pid, delta},
//                   clearing what they read; each adds its count to rec[H_L]
//   nlb             the header (survivors, kept / tail counts, last kept symbol)
//   (nlb, grid)     this rank's piece of the stale-window superset
template <typename S>
__global__ __launch_bounds__(TPB) void k_shard_send(DevState* st, uint32_t round, Table dt, const S* __restrict__ cur,
                                                    const S* __restrict__ oth, const uint32_t* __restrict__ hitmask,
                                                    const uint32_t* __restrict__ grpsum, uint32_t* __restrict__ rec,
                                                    uint32_t cap_list, uint32_t cap_win, uint32_t nlb) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (!merge_active(st, round)) {
        if (blockIdx.x == nlb && threadIdx.x < HDR) rec[threadIdx.x] = 0u;   // inactive round: ACTIVE = 0
        return;
    }
    if (blockIdx.x < nlb) {   // ── list role ──
        shard_list_role(st, dt, rec, cap_list, nlb);
        return;
    }
    const bool exact = (st->sharded & 2u) != 0;
    const uint32_t n = st->n, mc = st->mc;
    // the stale-window superset [gnew - mc, gnew) ∩ this rank's previous input stream
    uint32_t w = 0, src0 = 0;
    if (!exact) {
        const uint64_t hi = st->gnew, lo = hi >= mc ? hi - mc : 0;
        const uint64_t a0 = lo > st->poff ? lo : st->poff;
        const uint64_t pe = st->poff + st->pln;
        const uint64_t a1 = hi < pe ? hi : pe;
        if (a1 > a0) { w = (uint32_t)(a1 - a0); src0 = (uint32_t)(a0 - st->poff); }
    }
    if (blockIdx.x > nlb) {   // ── window role ──
        const uint32_t wc = w < cap_win ? w : cap_win;
        uint32_t* win = rec + HDR + 2 * (uint64_t)cap_list;
        const uint32_t nb = gridDim.x - nlb - 1, b = blockIdx.x - nlb - 1;
        for (uint32_t i = b * TPB + threadIdx.x; i < wc; i += nb * TPB) win[i] = to_canon<S>(oth[src0 + i]);
        return;
    }
    // ── header role ──
    __shared__ uint32_t wred[TPB / 64];
    const uint32_t ngrp = (uint32_t)gbpe_div_up(gbpe_div_up(n, TILE), GRP);
    uint32_t surv = 0;   // local survivors = sum of the group sums k_delta accumulated
    for (uint32_t g = threadIdx.x; g < ngrp; g += TPB) surv += grpsum[g * GSTR];
    for (int o = 32; o > 0; o >>= 1) surv += __shfl_xor(surv, o);
    if (lane == 0) wred[wid] = surv;
    __syncthreads();
    surv = 0;
    for (int k = 0; k < TPB / 64; ++k) surv += wred[k];
    if (wid != 0) return;
    // the last kept survivor: largest j < limit with hit(j) == 0, after the A-side rewrite
    const uint32_t limit = st->new_n < n ? st->new_n : n;
    int64_t wi = limit ? (int64_t)(limit - 1) / 32 : -1;
    uint32_t found = 0xFFFFFFFFu;
    while (wi >= 0 && found == 0xFFFFFFFFu) {
        const int64_t mywi = wi - lane;
        uint32_t inv = 0;
        if (mywi >= 0) inv = ~hitmask[mywi] & lane_mask32((uint64_t)mywi * 32, limit);
        const unsigned long long has = __ballot(inv != 0u);
        if (has) {
            const int l = __ffsll((long long)has) - 1;
            const uint32_t inv_l = __shfl(inv, l);
            found = (uint32_t)((wi - l) * 32 + (31 - __clz(inv_l)));
        }
        wi -= 64;
    }
    if (lane != 0) return;
    uint32_t last = 0;
    if (found != 0xFFFFFFFFu) {
        last = cur[found];
        const uint32_t f1 = found + 1;
        if (f1 < n && ((hitmask[f1 / 32] >> (f1 % 32)) & 1u)) last = st->nw | (last & Sym<S>::WS);
        last = to_canon<S>(last);
    }
    const uint32_t m_r = st->m;
    rec[H_ACTIVE] = 1u;
    rec[H_KEPT] = surv - m_r;
    rec[H_M] = m_r;
    rec[H_W] = w;
    rec[H_LASTSYM] = last;
    rec[H_HASLAST] = found != 0xFFFFFFFFu ? 1u : 0u;
    rec[H_SURV] = surv;
    rec[H_LN] = n;
    rec[H_MC] = mc;
    rec[H_A] = st->a;
    rec[H_B] = st->b;
    rec[H_ID] = st->nw;
    rec[H_DFULL] = st->dfull;   // an overflowed delta table: the list in this record is incomplete
    for (int k = H_DFULL + 1; k < HDR; ++k) rec[k] = 0u;
}

struct ShardView {   // per-WG decisions from the gathered headers (identical on every rank)
    uint32_t L[64], W[64], K[64];
    uint32_t lpre[65], wpre[65];
    uint32_t m, owner, x0, has_x0, overflow, bad, max_l, max_w, surv;
};

__device__ void shard_view(const DevState* st, const uint32_t* __restrict__ recv, uint32_t R, uint32_t rw,
                           uint32_t cap_list, uint32_t cap_win, ShardView& v) {
    if (threadIdx.x < 64) {
        const uint32_t q = threadIdx.x;
        const uint32_t* h = recv + (uint64_t)q * rw;
        const bool in = q < R;
        const uint32_t L = in ? h[H_L] : 0u, W = in ? h[H_W] : 0u, K = in ? h[H_KEPT] : 0u;
        const uint32_t M = in ? h[H_M] : 0u, S = in ? h[H_SURV] : 0u;
        const bool bad = in && (h[H_ACTIVE] != 1u || h[H_MC] != st->mc || h[H_A] != st->a || h[H_B] != st->b ||
                                h[H_ID] != st->nw);
        const bool dfull = in && h[H_DFULL] != 0u;
        const bool ovf = in && (L > cap_list || W > cap_win || dfull);
        uint32_t li = L, wi = W;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t a = __shfl_up(li, o), b = __shfl_up(wi, o);
            if ((int)q >= o) { li += a; wi += b; }
        }
        uint32_t m = M, surv = S, ml = dfull ? max(L, 4u * cap_list) : L, mw = W;
        for (int o = 32; o > 0; o >>= 1) {
            m += __shfl_xor(m, o);
            surv += __shfl_xor(surv, o);
            ml = max(ml, (uint32_t)__shfl_xor(ml, o));
            mw = max(mw, (uint32_t)__shfl_xor(mw, o));
        }
        const unsigned long long kept = __ballot(in && K > 0u);
        const unsigned long long ob = __ballot(ovf), bb = __ballot(bad);
        v.L[q] = L;
        v.W[q] = W;
        v.K[q] = K;
        v.lpre[q + 1] = li;
        v.wpre[q + 1] = wi;
        if (q == 0) {
            v.lpre[0] = 0u;
            v.wpre[0] = 0u;
            v.m = (st->sharded & 2u) ? 0u : m;
            v.surv = surv;
            v.overflow = ob != 0ull;
            v.bad = bb != 0ull;
            v.max_l = ml;
            v.max_w = mw;
            v.has_x0 = kept != 0ull;
            v.owner = kept ? 63u - (uint32_t)__clzll((long long)kept) : 0u;
            v.x0 = kept ? recv[(uint64_t)v.owner * rw + H_LASTSYM] : 0u;
        }
    }
    __syncthreads();
}

// symbol g of the gathered superset (pieces in rank order)
__device__ __forceinline__ uint32_t sup_at(const ShardView& v, const uint32_t* __restrict__ recv, uint32_t R,
                                           uint32_t rw, uint32_t cap_list, uint32_t g) {
    uint32_t q = 0;
    while (q + 1 < R && v.wpre[q + 1] <= g) ++q;
    return recv[(uint64_t)q * rw + HDR + 2 * cap_list + (g - v.wpre[q])];
}

// Phase-2 receive kernel, two block roles (after one all-gather of the records):
//   [0, nab)     every rank's count deltas + the stale window's pairs into the
//                replica; block 0 also commits the new global layout
//   [nab, grid)  the owner rank (last one that kept a survivor) appends the window
template <typename S>
__global__ __launch_bounds__(TPB) void k_shard_recv(DevState* st, uint32_t round, const uint32_t* __restrict__ recv,
                                                    uint32_t R, uint32_t cap_list, uint32_t cap_win, Table tb,
                                                    uint32_t cap_syms, S* __restrict__ oth, uint32_t nab) {
    __shared__ ShardView v;
    __shared__ LdsTab<LTAB> lt;
    if (!merge_active(st, round)) return;
    const uint32_t rw = HDR + 2 * cap_list + cap_win;
    shard_view(st, recv, R, rw, cap_list, cap_win, v);
    if (blockIdx.x >= nab) {   // ── append role ──
        if (v.bad || v.overflow || v.m == 0 || v.owner != st->rank) return;
        const uint32_t kept = v.K[st->rank];
        if ((uint64_t)kept + v.m + TILE > cap_syms) return;   // block 0 flags ERR_SHARD_CAPACITY
        const uint32_t g0 = v.wpre[R] - v.m, nb = gridDim.x - nab, b = blockIdx.x - nab;
        for (uint32_t j = b * TPB + threadIdx.x; j < v.m; j += nb * TPB)
            oth[kept + j] = (S)from_canon<S>(sup_at(v, recv, R, rw, cap_list, g0 + j));
        return;
    }
    if (v.bad) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { atomicOr(&st->err, ERR_SHARD_RECORD); st->stop = 1u; }
        return;
    }
    if (v.overflow) {   // stall on every rank: undo k_select's bookkeeping, ask the host for room
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const uint32_t pid = (st->a << 16) | st->b;
            const uint32_t idx = table_find(tb, pid);
            if (idx != 0xFFFFFFFFu) {
                tb.slots[idx].y = st->mc;
                tb.dirty[idx >> BLK_LOG2] = 1u;
            }
            st->next_id -= 1u;
            st->epoch -= 1u;
            st->merges_done -= 1u;
            st->stall = 1u;
            st->need_l = v.max_l;
            st->need_w = v.max_w;
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // new global layout
        uint64_t tot = 0, before = 0;
        uint32_t mine = 0;
        for (uint32_t q = 0; q < R; ++q) {
            const uint64_t nl = (uint64_t)v.K[q] + (q == v.owner ? v.m : 0u);
            if (q < st->rank) before += nl;
            if (q == st->rank) mine = (uint32_t)nl;
            tot += nl;
        }
        if (tot != st->gnew || (uint64_t)v.surv != st->gn - st->mc) {
            atomicOr(&st->err, ERR_SHARD_LAYOUT);
            st->need_l = (uint32_t)tot;      // diagnostics for the host message
            st->need_w = v.surv;
        }
        if ((uint64_t)mine + TILE > cap_syms) atomicOr(&st->err, ERR_SHARD_CAPACITY);
        st->owner = v.owner;
        st->m_glob = v.m;
        st->peak_l = max(st->peak_l, v.max_l);
        st->peak_w = max(st->peak_w, v.max_w);
        st->nl_next = mine;
        st->off_next = before;
        st->ln_last = (uint32_t)((uint64_t)v.K[R - 1] + (R - 1 == v.owner ? v.m : 0u));
    }
    // every rank's count deltas into the replica
    const uint32_t total = v.lpre[R];
    for (uint32_t e = blockIdx.x * TPB + threadIdx.x; e < total; e += nab * TPB) {
        uint32_t q = 0;
        while (q + 1 < R && v.lpre[q + 1] <= e) ++q;
        const uint32_t* l = recv + (uint64_t)q * rw + HDR + 2 * (e - v.lpre[q]);
        table_add(tb, st, l[0], l[1]);
    }
    // pairs of the stale window = last m symbols of the superset, after x0
    const uint32_t m = v.m;
    if (m <= blockIdx.x * TPB) return;   // no window symbols for this block (uniform)
    lds_clear(lt);
    __syncthreads();
    const uint32_t sup = v.wpre[R], g0 = sup - m;
    for (uint32_t j = blockIdx.x * TPB + threadIdx.x; j < m; j += nab * TPB) {
        uint32_t xp;
        if (j == 0) {
            if (!v.has_x0) continue;
            xp = v.x0;
        } else {
            xp = sup_at(v, recv, R, rw, cap_list, g0 + j - 1);
        }
        const uint32_t x = sup_at(v, recv, R, rw, cap_list, g0 + j);
        const uint32_t t0 = xp & 0xFFFFu, t1 = x & 0xFFFFu;
        if (!(x & 0x10000u) && t0 && t1) lds_add(lt, tb, st, (t0 << 16) | t1, 1u);
    }
    lds_flush(lt, tb, st);
}

// ── sector-sparse sharded loop ──
// Phase 1 is k_body on the local sectors (deltas into the per-merge delta table;
// the last rank also runs the zone, which carries the global stream's stale
// window) followed by k_shard_send_sp: the delta list and a header with the
// local length after the merge.  Phase 2, after the all-gather, is
// k_shard_apply_sp (every rank's deltas into the replica, the new global
// layout) and k_refresh (finish == 2).  Nothing crosses ranks but deltas and
// lengths: the zone rank is the only one whose pairs depend on the quirk.
__device__ __forceinline__ bool sp_round_active(const DevState* st, uint32_t round) {
    return !st->stop && !st->sp_abort && !st->stall && st->sel_round == round + 1u;
}

__global__ __launch_bounds__(TPB) void k_shard_send_sp(DevState* st, DevState* zst, uint32_t round, Table dt,
                                                       uint32_t* __restrict__ rec, uint32_t cap_list, uint32_t nlb) {
    if (!sp_round_active(st, round)) {
        if (blockIdx.x == nlb && threadIdx.x < HDR) rec[threadIdx.x] = 0u;   // inactive round: ACTIVE = 0
        return;
    }
    if (blockIdx.x < nlb) {
        shard_list_role(st, dt, rec, cap_list, nlb);
        return;
    }
    if (threadIdx.x != 0) return;
    const uint32_t zn = st->is_last && zst->valid_total ? zst->valid_total - 1u : 0u;   // zone survivors
    const uint32_t ln = (st->B - st->body_rm) + zn;   // local length after the merge
    st->new_n = ln;
    rec[H_ACTIVE] = 1u;
    rec[H_KEPT] = ln;
    rec[H_M] = 0u;
    rec[H_W] = 0u;
    rec[H_LASTSYM] = 0u;
    rec[H_HASLAST] = 0u;
    rec[H_SURV] = ln;
    rec[H_LN] = ln;
    rec[H_MC] = st->mc;
    rec[H_A] = st->a;
    rec[H_B] = st->b;
    rec[H_ID] = st->nw;
    rec[H_DFULL] = st->dfull;
    rec[H_ZN] = st->is_last ? zn : 0u;
    rec[H_ZM] = st->is_last ? zst->m : 0u;
}

__global__ __launch_bounds__(TPB) void k_shard_apply_sp(DevState* st, uint32_t round, const uint32_t* __restrict__ recv,
                                                        uint32_t R, uint32_t cap_list, uint32_t cap_win, Table tb,
                                                        uint32_t nab) {
    __shared__ ShardView v;
    if (!sp_round_active(st, round)) return;
    const uint32_t rw = HDR + 2 * cap_list + cap_win;
    shard_view(st, recv, R, rw, cap_list, cap_win, v);
    if (v.bad || v.overflow) {   // records disagree, or a list did not fit (k_body's bound should prevent it)
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            atomicOr(&st->err, v.bad ? ERR_SHARD_RECORD : ERR_SHARD_CAPACITY);
            st->stop = 1u;
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // new global layout (rank order)
        uint64_t tot = 0, before = 0;
        uint32_t mine = 0, zm = 0;
        for (uint32_t q = 0; q < R; ++q) {
            const uint32_t nl = recv[(uint64_t)q * rw + H_LN];
            if (q < st->rank) before += nl;
            if (q == st->rank) mine = nl;
            tot += nl;
            zm += recv[(uint64_t)q * rw + H_ZM];
        }
        if (tot != st->gn - st->mc || mine != st->new_n) {
            atomicOr(&st->err, ERR_SHARD_LAYOUT);
            st->need_l = (uint32_t)tot;
            st->need_w = mine;
        }
        st->m_glob = zm;
        st->peak_l = max(st->peak_l, max(v.max_l, 6u * st->mc + 64u));   // what k_body's stall bound asks for
        st->poff = st->off;
        st->pln = st->n;
        st->off = before;
        st->gn = tot;
        st->ln_last = recv[(uint64_t)(R - 1) * rw + H_LN];
        st->zlast = recv[(uint64_t)(R - 1) * rw + H_ZN];
    }
    const uint32_t total = v.lpre[R];   // every rank's count deltas into the replica
    for (uint32_t e = blockIdx.x * TPB + threadIdx.x; e < total; e += nab * TPB) {
        uint32_t q = 0;
        while (q + 1 < R && v.lpre[q + 1] <= e) ++q;
        const uint32_t* l = recv + (uint64_t)q * rw + HDR + 2 * (e - v.lpre[q]);
        table_add(tb, st, l[0], l[1]);
    }
}

__global__ void k_add_list(DevState* st, Table tb, const uint2* __restrict__ list, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && list[i].x && list[i].y) table_add(tb, st, list[i].x, list[i].y);
}

__global__ void k_dump_list(Table tb, uint2* __restrict__ out, uint32_t* __restrict__ nout, uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > tb.mask) return;
    const uint2 e = tb.slots[i];
    if (e.x && (int32_t)e.y > 0) {
        const uint32_t k = atomicAdd(nout, 1u);
        if (k < cap) out[k] = e;
    }
}

}  // namespace

// ─── sharded host API ───────────────────────────────────────────────────────

namespace {
inline uint32_t shard_record_words(uint32_t cl, uint32_t cw) { return HDR + 2 * cl + cw; }
}  // namespace

extern "C" int gbpe_shard_create(gbpe_ctx* ctx, const uint8_t* bytes, uint64_t n, const uint8_t* word_starts,
                                 int input_on_device, const gbpe_train_opts* opts, uint32_t rank, uint32_t world,
                                 uint64_t cap_extra, gbpe_trainer** out) {
    if (!ctx || !out || !opts) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    if (world == 0 || world > 64 || rank >= world) return gbpe_set_error(ctx, GBPE_E_INVALID, "rank/world out of range (world <= 64)");
    // the replica holds GLOBAL counts and is only ever rehashed at its size: size
    // it for the corpus as a whole (shard_rehash; no growth path)
    gbpe_train_opts o = *opts;
    if (o.table_log2 == 0) {
        const uint64_t gn = n * world;
        o.table_log2 = gn > (512ull << 20) ? 24u : gn > (64ull << 20) ? 23u : 22u;
    }
    int rc = trainer_create_impl(ctx, bytes, n, word_starts, input_on_device, &o, cap_extra, out);
    if (rc != GBPE_OK) return rc;
    gbpe_trainer* t = *out;
    t->sharded = true;
    t->rank = rank;
    t->world = world;
    t->dt.mask = t->tb.mask;
    t->dt.nblk = t->tb.nblk;
    t->dt.used = nullptr;   // every key is new each merge: no shared counter on the state line
    t->dt.full = &t->st->dfull;
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    hipStream_t s = ctx->stream;
    if (hipMalloc(&t->dt.slots, slots * sizeof(uint2)) != hipSuccess ||
        hipMalloc(&t->dt.dirty, t->dt.nblk * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t->d_nlog, (size_t)t->batch * sizeof(uint32_t)) != hipSuccess ||
        hipHostMalloc((void**)&t->h_nlog, (size_t)t->batch * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
        gbpe_trainer_destroy(t);
        *out = nullptr;
        return gbpe_set_error(ctx, GBPE_E_OOM, "hipMalloc(shard buffers) failed");
    }
    t->h_st->sharded = 1u | ((t->flags & GBPE_TRAIN_EXACT_COMPACTION) ? 2u : 0u);
    t->h_st->rank = rank;
    t->h_st->world = world;
    if (hipMemsetAsync(t->dt.slots, 0, slots * sizeof(uint2), s) != hipSuccess ||
        hipMemsetAsync(t->dt.dirty, 0, t->dt.nblk * sizeof(uint32_t), s) != hipSuccess ||
        hipMemcpyAsync(&t->st->sharded, &t->h_st->sharded, 3 * sizeof(uint32_t), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        gbpe_trainer_destroy(t);
        *out = nullptr;
        return gbpe_set_error(ctx, GBPE_E_DEVICE, "shard init failed");
    }
    return GBPE_OK;
}

extern "C" int gbpe_shard_global_len(gbpe_trainer* t, uint64_t* gn) {
    if (!t || !gn || !t->sharded) return GBPE_E_INVALID;
    *gn = t->h_st->gn;
    return GBPE_OK;
}

extern "C" int gbpe_shard_local_len(gbpe_trainer* t, uint64_t* n) {
    if (!t || !n) return GBPE_E_INVALID;
    *n = t->n;
    return GBPE_OK;
}

extern "C" int gbpe_shard_set_layout(gbpe_trainer* t, const uint64_t* lens, uint32_t world) {
    if (!t || !lens || !t->sharded || world != t->world) return t ? gbpe_set_error(t->ctx, GBPE_E_INVALID, "set_layout: bad arguments") : GBPE_E_INVALID;
    if (lens[t->rank] != t->n) return gbpe_set_error(t->ctx, GBPE_E_INVALID, "set_layout: own length mismatch");
    uint64_t gn = 0, off = 0;
    for (uint32_t q = 0; q < world; ++q) {
        if (q < t->rank) off += lens[q];
        gn += lens[q];
    }
    if (gn >= 0xFFFFFFFFFFull) return gbpe_set_error(t->ctx, GBPE_E_INVALID, "global corpus too large");
    DevState* hs = t->h_st;
    hs->gn = gn;
    hs->off = off;
    hs->poff = off;      // the previous input stream before merge 1: the zeroed ping-pong buffer
    hs->pln = t->n;
    hipStream_t s = t->ctx->stream;
    const size_t o = offsetof(DevState, sharded);   // only the shard section: the rest lives on the device
    TR_HIP(t, hipMemcpyAsync((char*)t->st + o, (char*)hs + o, sizeof(DevState) - o, hipMemcpyHostToDevice, s));
    TR_HIP(t, hipStreamSynchronize(s));
    return GBPE_OK;
}

extern "C" int gbpe_shard_export_counts(gbpe_trainer* t, void* d_out, uint64_t cap, uint64_t* n_pairs) {
    if (!t || !n_pairs) return GBPE_E_INVALID;
    hipStream_t s = t->ctx->stream;
    uint32_t* d_cnt = nullptr;
    TR_HIP(t, hipMalloc(&d_cnt, sizeof(uint32_t)));
    hipError_t e = hipMemsetAsync(d_cnt, 0, sizeof(uint32_t), s);
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    hipLaunchKernelGGL(k_dump_list, dim3((uint32_t)gbpe_div_up(slots, 256)), dim3(256), 0, s, t->tb, (uint2*)d_out,
                       d_cnt, d_out ? (uint32_t)cap : 0u);
    uint32_t cnt = 0;
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(&cnt, d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(d_cnt);
    if (e != hipSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "export_counts failed: %s", hipGetErrorString(e));
    *n_pairs = cnt;
    if (d_out && cnt > cap) return gbpe_set_error(t->ctx, GBPE_E_CAPACITY, "export_counts: need %u", cnt);
    return GBPE_OK;
}

extern "C" int gbpe_shard_import_counts(gbpe_trainer* t, const void* d_lists, const uint64_t* counts, uint32_t world,
                                        uint64_t stride) {
    if (!t || !d_lists || !counts || world != t->world) return t ? gbpe_set_error(t->ctx, GBPE_E_INVALID, "import_counts: bad arguments") : GBPE_E_INVALID;
    hipStream_t s = t->ctx->stream;
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    TR_HIP(t, hipMemsetAsync(t->tb.slots, 0, slots * sizeof(uint2), s));
    TR_HIP(t, hipMemsetAsync(t->tb.bmax, 0, (uint64_t)t->tb.nblk * sizeof(uint64_t), s));
    TR_HIP(t, hipMemsetAsync(t->tb.blive, 0, (uint64_t)t->tb.nblk * sizeof(uint32_t), s));
    TR_HIP(t, hipMemsetAsync(&t->st->used, 0, sizeof(uint32_t), s));
    const uint2* base = (const uint2*)d_lists;
    for (uint32_t q = 0; q < world; ++q) {
        if (counts[q] == 0) continue;
        hipLaunchKernelGGL(k_add_list, dim3((uint32_t)gbpe_div_up(counts[q], 256)), dim3(256), 0, s, t->st, t->tb,
                           base + q * stride, counts[q]);
    }
    hipLaunchKernelGGL(k_clear_dirty_all, dim3((uint32_t)gbpe_div_up(t->tb.nblk, 256)), dim3(256), 0, s, t->st, t->tb);
    if (t->u16)
        hipLaunchKernelGGL(k_refresh<uint16_t>, dim3(grid_blocks(t->ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st,
                           0u, 0, t->tb, (uint16_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    else
        hipLaunchKernelGGL(k_refresh<uint32_t>, dim3(grid_blocks(t->ctx, t->tb.nblk, 4)), dim3(TPB), 0, s, t->st,
                           0u, 0, t->tb, (uint32_t*)nullptr, (const uint32_t*)nullptr, (DevState*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    TR_HIP(t, hipMemcpyAsync(t->h_st, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (t->h_st->err) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "import_counts: table error 0x%x", t->h_st->err);
    return GBPE_OK;
}

namespace {
// rebuild a crowded replica without the stream (the table holds GLOBAL counts)
int shard_rehash(gbpe_trainer* t) {
    uint64_t P = 0;
    int rc = gbpe_shard_export_counts(t, nullptr, 0, &P);
    if (rc != GBPE_OK) return rc;
    void* d = nullptr;
    TR_HIP(t, hipMalloc(&d, (P + 1) * sizeof(uint2)));
    rc = gbpe_shard_export_counts(t, d, P, &P);
    if (rc == GBPE_OK) {
        const uint64_t cnt[1] = {P};
        const uint32_t w = t->world;
        t->world = 1;   // import a single list
        rc = gbpe_shard_import_counts(t, d, cnt, 1, 0);
        t->world = w;
    }
    hipFree(d);
    return rc;
}
}  // namespace

extern "C" int gbpe_shard_record_words(uint32_t cap_list, uint32_t cap_win) {
    return (int)shard_record_words(cap_list, cap_win);
}

extern "C" int gbpe_shard_step_begin(gbpe_trainer* t, uint32_t max_merges) {
    if (!t || !t->sharded) return GBPE_E_INVALID;
    uint32_t k = max_merges ? max_merges : t->batch;
    if (k > t->batch) k = t->batch;
    if (t->done + k > t->needed) k = t->needed - t->done;
    t->step_k = t->stop ? 0u : k;
    if (t->step_k == 0) return GBPE_OK;
    const uint64_t slots = (uint64_t)t->tb.mask + 1;
    if ((uint64_t)t->h_st->used * 2 > slots) {   // identical on every rank (replica tables)
        int rc = sp_exit_any(t);
        if (rc == GBPE_OK) rc = shard_rehash(t);
        if (rc != GBPE_OK) return rc;
    }
    DevState* hs = t->h_st;
    // sector-sparse loop: decided from global state only, so every rank
    // enters together; the last rank holds the zone, which must fit one workgroup
    if (t->sp_cooldown) {
        --t->sp_cooldown;
    } else if (!t->sp && !(t->flags & GBPE_TRAIN_DENSE_ONLY) && t->last_mc && hs->ln_last) {
        const uint64_t zt = (uint64_t)t->sp_zt * t->last_mc + 64;
        const uint32_t zmax = t->u16 ? zone_max<uint16_t>(1024) : zone_max<uint32_t>(1024);
        if (((t->flags & GBPE_TRAIN_SPARSE_EARLY) || (uint64_t)t->last_mc * t->sp_div <= hs->gn) &&
            2 * zt + 4096 <= zmax && (uint64_t)hs->ln_last >= 4 * zt) {
            const bool last = t->rank + 1 == t->world;
            int rc = t->u16 ? sp_enter<uint16_t>(t, last) : sp_enter<uint32_t>(t, last);
            if (rc != GBPE_OK) return rc;
            if (!t->sp) return gbpe_set_error(t->ctx, GBPE_E_INTERNAL, "sharded sparse entry failed on rank %u", t->rank);
        }
    }
    if (t->sp) {
        int rc = t->u16 ? sp_shrink<uint16_t>(t) : sp_shrink<uint32_t>(t);
        if (rc == GBPE_OK && t->sp_age >= 4096) {
            const bool wb = t->sp_bits_age >= 16384;
            rc = t->u16 ? sp_filters<uint16_t>(t, wb) : sp_filters<uint32_t>(t, wb);
        }
        if (rc != GBPE_OK) return rc;
        hs->sel_round = 0;
        TR_HIP(t, hipMemcpyAsync(&t->st->sel_round, &hs->sel_round, sizeof(uint32_t), hipMemcpyHostToDevice,
                                 t->ctx->stream));
    }
    hs->merges_done = 0;
    hs->budget = t->step_k;
    hs->stall = 0;
    hs->peak_l = hs->peak_w = 0;
    hipStream_t s = t->ctx->stream;
    TR_HIP(t, hipMemcpyAsync(&t->st->merges_done, &hs->merges_done, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->st->budget, &hs->budget, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->st->stall, &hs->stall, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    TR_HIP(t, hipMemcpyAsync(&t->st->peak_l, &hs->peak_l, 2 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    return GBPE_OK;
}

namespace {
// the per-merge delta table only has to hold one merge's distinct deltas: size it
// 4x the record's list capacity (>= 2 blocks) so k_shard_send scans few blocks
Table delta_view(const gbpe_trainer* t, uint32_t cl) {
    Table d = t->dt;
    uint64_t want = 4ull * cl, sl = 1ull << (BLK_LOG2 + 1);
    while (sl < want && sl < (uint64_t)t->dt.mask + 1) sl <<= 1;
    d.mask = (uint32_t)(sl - 1);
    d.nblk = (uint32_t)(sl >> BLK_LOG2);
    return d;
}

template <typename S>
int shard_phase1(gbpe_trainer* t, uint32_t round, uint32_t* rec, uint32_t cl, uint32_t cw) {
    hipStream_t s = t->ctx->stream;
    S* cur = (S*)t->buf[t->cur ^ (round & 1)];
    S* oth = (S*)t->buf[t->cur ^ (round & 1) ^ 1];
    const uint32_t eager = (uint32_t)gbpe_div_up(t->n, TILE);   // the stream may grow by appended windows
    const uint32_t g_delta = (uint32_t)gbpe_div_up(t->cap_syms, TILE) - 1;
    const Table dt = delta_view(t, cl);
    hipLaunchKernelGGL(k_select, dim3(1), dim3(SEL_THREADS), 0, s, t->st, t->tb, t->d_log, t->grpsum, t->d_nlog, rec,
                       (DevState*)nullptr, 0u);
    if (t->flags & GBPE_TRAIN_EXACT_COMPACTION)
        hipLaunchKernelGGL((k_delta<S, true>), dim3(g_delta), dim3(TPB), 0, s, t->st, round, (const S*)cur, dt,
                           t->hitmask, t->tile_cnt, t->grpsum, eager);
    else
        hipLaunchKernelGGL((k_delta<S, false>), dim3(g_delta), dim3(TPB), 0, s, t->st, round, (const S*)cur, dt,
                           t->hitmask, t->tile_cnt, t->grpsum, eager);
    const uint32_t nlb = grid_blocks(t->ctx, dt.nblk, 2);
    const uint32_t nwb = grid_persistent(t->ctx, gbpe_div_up(cw, TPB * 8) + 1, 1);
    hipLaunchKernelGGL(k_shard_send<S>, dim3(nlb + 1 + nwb), dim3(TPB), 0, s, t->st, round, dt, (const S*)cur,
                       (const S*)oth, (const uint32_t*)t->hitmask, (const uint32_t*)t->grpsum, rec, cl, cw, nlb);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

template <typename S>
int shard_phase2(gbpe_trainer* t, uint32_t round, const uint32_t* recv, uint32_t cl, uint32_t cw) {
    hipStream_t s = t->ctx->stream;
    S* cur = (S*)t->buf[t->cur ^ (round & 1)];
    S* oth = (S*)t->buf[t->cur ^ (round & 1) ^ 1];
    const uint32_t R = t->world;
    const uint32_t g_tiles = (uint32_t)gbpe_div_up(t->cap_syms, TILE) - 1;
    const uint32_t cap = (uint32_t)t->cap_syms;
    const uint32_t nab = grid_persistent(t->ctx, 1u << 20, 2), npb = grid_persistent(t->ctx, 1u << 20, 1);
    hipLaunchKernelGGL(k_shard_recv<S>, dim3(nab + npb), dim3(TPB), 0, s, t->st, round, recv, R, cl, cw, t->tb, cap, oth,
                       nab);
    if (t->flags & GBPE_TRAIN_EXACT_COMPACTION)
        hipLaunchKernelGGL((k_compact<S, true>), dim3(g_tiles), dim3(CTPB), 0, s, t->st, round, cur, oth,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb);
    else
        hipLaunchKernelGGL((k_compact<S, false>), dim3(g_tiles), dim3(CTPB), 0, s, t->st, round, cur, oth,
                           (const uint32_t*)t->hitmask, (const uint32_t*)t->tile_cnt, (const uint32_t*)t->grpsum, t->tb);
    hipLaunchKernelGGL(k_refresh<S>, dim3(grid_blocks(t->ctx, t->tb.nblk, 2)), dim3(TPB), 0, s, t->st, round, 1,
                       t->tb, cur, (const uint32_t*)nullptr, (DevState*)nullptr);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}
}  // namespace

namespace {
// sector-sparse sharded merge, phase 1: k_body (deltas into the per-merge delta
// table; the zone on the last rank) + k_shard_send_sp
template <typename S>
int shard_phase1_sp(gbpe_trainer* t, uint32_t round, uint32_t* rec, uint32_t cl) {
    hipStream_t s = t->ctx->stream;
    S* zc = (S*)t->zbuf[t->zcur ^ (round & 1)];
    S* zo = (S*)t->zbuf[t->zcur ^ (round & 1) ^ 1];
    const bool exact = (t->flags & GBPE_TRAIN_EXACT_COMPACTION) != 0;
    const Table dt = delta_view(t, cl);
    const bool zone = t->h_st->is_last != 0;
    const uint32_t zn = zone ? t->n - t->h_st->B : 0u;   // the zone only shrinks within a step
    const int bt = zn <= (t->u16 ? zone_max<uint16_t>(256) : zone_max<uint32_t>(256)) ? 256 : 1024;
    uint32_t nbody = 0, wpg = 0;
    body_grid(t, bt, &nbody, &wpg);
    SelShard sh;
    sh.cap_list = cl;
    sh.zmax = t->u16 ? zone_max<uint16_t>(1024) : zone_max<uint32_t>(1024);
    sh.nlog = t->d_nlog;
    sh.rec = rec;
    const uint32_t gb = nbody + (zone ? 1u : 0u);
    if (exact)
        launch_body<S, true>(bt, gb, s, t->st, round, (S*)sp_body(t), t->sec, t->bits, t->W, wpg, t->sig, t->tb, nbody,
                             (const S*)zo, (S*)t->wtmp, 0u, t->zst, zc, zone ? 1u : 0u, (const uint64_t*)t->part,
                             t->g_refresh, t->d_log, t->grpsum, t->wg_bytes, dt, sh, sp_mul(t));
    else
        launch_body<S, false>(bt, gb, s, t->st, round, (S*)sp_body(t), t->sec, t->bits, t->W, wpg, t->sig, t->tb, nbody,
                              (const S*)zo, (S*)t->wtmp, 0u, t->zst, zc, zone ? 1u : 0u, (const uint64_t*)t->part,
                              t->g_refresh, t->d_log, t->grpsum, t->wg_bytes, dt, sh, sp_mul(t));
    const uint32_t nlb = grid_blocks(t->ctx, dt.nblk, 2);
    hipLaunchKernelGGL(k_shard_send_sp, dim3(nlb + 1), dim3(TPB), 0, s, t->st, t->zst, round, dt, rec, cl, nlb);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}

// phase 2: every rank's deltas into the replica, the new layout, then k_refresh
template <typename S>
int shard_phase2_sp(gbpe_trainer* t, uint32_t round, const uint32_t* recv, uint32_t cl, uint32_t cw) {
    hipStream_t s = t->ctx->stream;
    const uint32_t nab = grid_persistent(t->ctx, 1u << 20, 2);
    hipLaunchKernelGGL(k_shard_apply_sp, dim3(nab), dim3(TPB), 0, s, t->st, round, recv, t->world, cl, cw, t->tb, nab);
    hipLaunchKernelGGL(k_refresh<S>, dim3(t->g_refresh), dim3(TPB), 0, s, t->st, round, 2, t->tb, (S*)nullptr,
                       (const uint32_t*)nullptr, t->zst, (uint32_t*)nullptr, FusedSel(), t->part);
    GBPE_LAUNCH_CHECK(t->ctx);
    return GBPE_OK;
}
}  // namespace

extern "C" int gbpe_shard_phase1(gbpe_trainer* t, uint32_t round, void* d_send, uint32_t cap_list, uint32_t cap_win) {
    if (!t || !t->sharded || !d_send) return GBPE_E_INVALID;
    if (round >= t->batch) return gbpe_set_error(t->ctx, GBPE_E_INVALID, "round out of range");
    if (round >= t->step_k) {   // nothing to do this round, but the record must say so
        TR_HIP(t, hipMemsetAsync(d_send, 0, HDR * sizeof(uint32_t), t->ctx->stream));
        return GBPE_OK;
    }
    if (t->sp)
        return t->u16 ? shard_phase1_sp<uint16_t>(t, round, (uint32_t*)d_send, cap_list)
                      : shard_phase1_sp<uint32_t>(t, round, (uint32_t*)d_send, cap_list);
    return t->u16 ? shard_phase1<uint16_t>(t, round, (uint32_t*)d_send, cap_list, cap_win)
                  : shard_phase1<uint32_t>(t, round, (uint32_t*)d_send, cap_list, cap_win);
}

extern "C" int gbpe_shard_phase2(gbpe_trainer* t, uint32_t round, const void* d_recv, uint32_t cap_list,
                                 uint32_t cap_win) {
    if (!t || !t->sharded || !d_recv) return GBPE_E_INVALID;
    if (round >= t->step_k) return GBPE_OK;
    if (t->sp)
        return t->u16 ? shard_phase2_sp<uint16_t>(t, round, (const uint32_t*)d_recv, cap_list, cap_win)
                      : shard_phase2_sp<uint32_t>(t, round, (const uint32_t*)d_recv, cap_list, cap_win);
    return t->u16 ? shard_phase2<uint16_t>(t, round, (const uint32_t*)d_recv, cap_list, cap_win)
                  : shard_phase2<uint32_t>(t, round, (const uint32_t*)d_recv, cap_list, cap_win);
}

extern "C" int gbpe_shard_step_end(gbpe_trainer* t, uint32_t* merges_out, uint32_t* n_done, uint32_t* early_stop,
                                   uint32_t* stalled, uint32_t* need_list, uint32_t* need_win) {
    if (!t || !t->sharded) return GBPE_E_INVALID;
    if (n_done) *n_done = 0;
    if (stalled) *stalled = 0;
    if (need_list) *need_list = 0;
    if (need_win) *need_win = 0;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    if (t->step_k == 0) return GBPE_OK;
    hipStream_t s = t->ctx->stream;
    DevState* hs = t->h_st;
    TR_HIP(t, hipMemcpyAsync(hs, t->st, sizeof(DevState), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipMemcpyAsync(t->h_log, t->d_log, (size_t)t->step_k * 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipMemcpyAsync(t->h_nlog, t->d_nlog, (size_t)t->step_k * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    TR_HIP(t, hipStreamSynchronize(s));
    if (hs->err) {
        return gbpe_set_error(t->ctx, (hs->err & ERR_SHARD_CAPACITY) ? GBPE_E_CAPACITY : GBPE_E_INTERNAL,
                              "sharded training invariant violated (err=0x%x: %s%s%s%s%s; merge %u, n %u, gn %llu, "
                              "gnew %llu, mc %u, new len total %u, survivors %u)", hs->err,
                              (hs->err & ERR_TABLE_FULL) ? "pair table full " : "",
                              (hs->err & ERR_PAIR_MISSING) ? "selected pair missing " : "",
                              (hs->err & ERR_SHARD_CAPACITY) ? "shard buffer too small for appended windows " : "",
                              (hs->err & ERR_SHARD_RECORD) ? "exchange records disagree " : "",
                              (hs->err & ERR_SHARD_LAYOUT) ? "gathered totals do not add up" : "",
                              t->done + hs->merges_done, hs->n, (unsigned long long)hs->gn,
                              (unsigned long long)hs->gnew, hs->mc, hs->need_l, hs->need_w);
    }
    const uint32_t done = hs->merges_done;
    // local algorithmic stream bytes s * (2 N_i + N_{i+1}) with the local lengths
    for (uint32_t r = 0; r < done; ++r) {
        const uint64_t N = t->h_nlog[r];
        const uint64_t N1 = r + 1 < done ? t->h_nlog[r + 1] : hs->n;
        t->bytes_moved += (uint64_t)t->bps * (2 * N + N1);
        if (merges_out) memcpy(merges_out + 4 * r, t->h_log + 4 * r, 4 * sizeof(uint32_t));
    }
    t->n = hs->n;
    if (done) t->last_mc = t->h_log[(done - 1) * 4 + 3];
    if (t->sp) {
        t->zcur ^= (int)(done & 1u);
        t->sp_merges += done;
        t->sp_age += done;
        t->sp_bits_age += done;
    } else {
        t->cur ^= (done & 1u);
    }
    t->done += done;
    t->stop = hs->stop != 0;
    t->step_k = 0;
    if (t->sp && hs->sp_abort) {   // the zone outgrew its bounds on the last rank: every rank goes dense
        int rc = sp_exit_any(t);
        if (rc != GBPE_OK) return rc;
        t->sp_cooldown = 1;
    }
    if (n_done) *n_done = done;
    if (early_stop) *early_stop = t->stop ? 1u : 0u;
    if (stalled) *stalled = hs->stall;
    // a stalled step reports what the stalled merge needs; otherwise the step's peaks
    if (need_list) *need_list = hs->stall ? hs->need_l : hs->peak_l;
    if (need_win) *need_win = hs->stall ? hs->need_w : hs->peak_w;
    return GBPE_OK;
}

// ─── native exchange: RCCL all-gather on the trainer's own stream ───────────
//
// The host loop of gpubpe/sharded.py issues three calls per merge (phase 1,
// torch all-gather, phase 2) and pays a cross-stream event wait per merge.
// gbpe_shard_step_comm runs the same protocol for a whole step inside the
// library: phase-1 kernels, ncclAllGather, phase-2 kernels, all enqueued on one
// stream with no host involvement.  RCCL is opened at run time (dlopen of
// librccl.so.1: the copy torch already loaded, or ROCm's), so the library has
// no link-time RCCL dependency.

#include <dlfcn.h>
#include <rccl/rccl.h>

struct gbpe_comm {
    ncclComm_t comm = nullptr;
    int device = 0;
    uint32_t rank = 0, world = 1;
};

namespace {
struct RcclApi {
    bool ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
};

RcclApi& rccl() {
    static RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            a.err = dlerror() ? dlerror() : "dlopen(librccl.so.1) failed";
            return a;
        }
        a.get_id = (decltype(a.get_id))dlsym(h, "ncclGetUniqueId");
        a.init = (decltype(a.init))dlsym(h, "ncclCommInitRank");
        a.destroy = (decltype(a.destroy))dlsym(h, "ncclCommDestroy");
        a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
        a.errstr = (decltype(a.errstr))dlsym(h, "ncclGetErrorString");
        a.ok = a.get_id && a.init && a.destroy && a.all_gather && a.errstr;
        if (!a.ok) a.err = "librccl.so.1 lacks the nccl* entry points";
        return a;
    }();
    return api;
}
}  // namespace

extern "C" int gbpe_comm_unique_id(uint8_t* out, uint32_t len) {
    if (!out || len < NCCL_UNIQUE_ID_BYTES) return GBPE_E_INVALID;
    RcclApi& r = rccl();
    if (!r.ok) return GBPE_E_DEVICE;
    ncclUniqueId id;
    if (r.get_id(&id) != ncclSuccess) return GBPE_E_DEVICE;
    memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return GBPE_OK;
}

extern "C" int gbpe_comm_create(gbpe_ctx* ctx, const uint8_t* id, uint32_t len, uint32_t rank, uint32_t world,
                                gbpe_comm** out) {
    if (!ctx || !id || !out || len < NCCL_UNIQUE_ID_BYTES || world == 0 || rank >= world)
        return gbpe_set_error(ctx, GBPE_E_INVALID, "comm_create: bad arguments");
    *out = nullptr;
    RcclApi& r = rccl();
    if (!r.ok) return gbpe_set_error(ctx, GBPE_E_DEVICE, "RCCL unavailable: %s", r.err.c_str());
    GBPE_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId uid;
    memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    auto* c = new (std::nothrow) gbpe_comm();
    if (!c) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    ncclResult_t e = r.init(&c->comm, (int)world, uid, (int)rank);
    if (e != ncclSuccess) {
        delete c;
        return gbpe_set_error(ctx, GBPE_E_DEVICE, "ncclCommInitRank: %s", r.errstr(e));
    }
    c->device = ctx->device;
    c->rank = rank;
    c->world = world;
    *out = c;
    return GBPE_OK;
}

extern "C" void gbpe_comm_destroy(gbpe_comm* c) {
    if (!c) return;
    if (c->comm && rccl().ok) rccl().destroy(c->comm);
    delete c;
}

extern "C" int gbpe_shard_step_comm(gbpe_trainer* t, gbpe_comm* comm, uint32_t max_merges, uint32_t cap_list,
                                    uint32_t cap_win, uint32_t* merges_out, uint32_t* n_done, uint32_t* early_stop,
                                    uint32_t* stalled, uint32_t* need_list, uint32_t* need_win) {
    if (!t || !t->sharded || !comm || comm->world != t->world || comm->rank != t->rank)
        return t ? gbpe_set_error(t->ctx, GBPE_E_INVALID, "step_comm: trainer / communicator mismatch") : GBPE_E_INVALID;
    int rc = gbpe_shard_step_begin(t, max_merges);
    if (rc != GBPE_OK) return rc;
    const uint64_t rw = shard_record_words(cap_list, cap_win);
    if (t->rec_words < rw) {   // library-owned exchange records (grow only)
        hipStream_t s0 = t->ctx->stream;
        TR_HIP(t, hipStreamSynchronize(s0));
        hipFree(t->rec_send);
        hipFree(t->rec_recv);
        t->rec_send = t->rec_recv = nullptr;
        t->rec_words = 0;
        TR_HIP(t, hipMalloc(&t->rec_send, rw * sizeof(uint32_t)));
        TR_HIP(t, hipMalloc(&t->rec_recv, rw * t->world * sizeof(uint32_t)));
        t->rec_words = rw;
    }
    hipStream_t s = t->ctx->stream;
    for (uint32_t k = 0; k < t->step_k; ++k) {
        rc = gbpe_shard_phase1(t, k, t->rec_send, cap_list, cap_win);
        if (rc != GBPE_OK) return rc;
        const ncclResult_t e = rccl().all_gather(t->rec_send, t->rec_recv, rw, ncclUint32, comm->comm, s);
        if (e != ncclSuccess) return gbpe_set_error(t->ctx, GBPE_E_DEVICE, "ncclAllGather: %s", rccl().errstr(e));
        rc = gbpe_shard_phase2(t, k, t->rec_recv, cap_list, cap_win);
        if (rc != GBPE_OK) return rc;
    }
    return gbpe_shard_step_end(t, merges_out, n_done, early_stop, stalled, need_list, need_win);
}
