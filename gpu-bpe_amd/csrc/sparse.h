// Sector-sparse merge loop: the word-lexicon body's sectors,
// token bitmap and pair signatures, the one-workgroup zone pass, and k_body — the
// per-merge pass over the candidate sectors.  Shares train_dev.h's state, pair
// table and LDS delta tables.
#pragma once

#include "train_dev.h"

namespace {

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
constexpr uint32_t SP_SHRINKS = 64;  // zone shrinks per sparse entry the first sector capacity allows for (sp_reserve grows it)
constexpr uint32_t SP_SHRINKS_MAX = 1024;   // zone shrinks per sparse entry

// Per-sector pair signature: a 2048-bit Bloom filter (3 hash bits) of every pair
// the sector has held since the filters were last rebuilt.  The token bitmap
// gives candidate sectors; the signature drops most of those where a and b are
// both present but never adjacent.  (1024 bits / 2 hash bits let through 5 of
// every 6 candidates without a site in the middle merges — a sector holds ~200
// pairs plus those its merges add — and every false candidate costs a sector
// pass: 2048 / 3 cuts that rate to a few percent.)
constexpr uint32_t SP_SIGW = 64;     // u32 words per sector signature
#ifdef GBPE_SIG_GLOBAL
constexpr bool SIG_LDS = false;      // (A/B build: every created pair's bits straight to the global signature)
#else
constexpr bool SIG_LDS = true;       // k_body gathers a sector's new signature bits in LDS (body_sector's lsig)
#endif
constexpr uint32_t SP_SIGB = SP_SIGW * 32 - 1;
__device__ __forceinline__ uint32_t sig_hash(uint32_t pid) { return gbpe_fmix32(pid ^ 0x9E3779B9u); }
#ifdef GBPE_SIG_SPREAD
// (A/B build: the three bits anywhere in the 2048 — a test loads up to three
// words on two 128-B lines)
__device__ __forceinline__ void sig_bits(uint32_t pid, uint32_t& b1, uint32_t& b2, uint32_t& b3) {
    const uint32_t h = sig_hash(pid), h2 = h * 0x9E3779B1u;
    b1 = h & SP_SIGB;
    b2 = (h >> 16) & SP_SIGB;
    b3 = (h2 >> 21) & SP_SIGB;
}
__device__ __forceinline__ bool sig_has(const uint32_t* __restrict__ sig, uint32_t pid) {
    uint32_t b1, b2, b3;
    sig_bits(pid, b1, b2, b3);
    return ((sig[b1 >> 5] >> (b1 & 31u)) & (sig[b2 >> 5] >> (b2 & 31u)) & (sig[b3 >> 5] >> (b3 & 31u)) & 1u) != 0u;
}
#else
// Blocked: the hash picks one 64-bit word of the 32, and the three bits inside
// it, so a candidate test is ONE 8-byte load (one line) instead of up to three
// words on two lines (the filter's false-positive rate at ~300 pairs per sector
// moves from ~4.6 % to ~5.5 %: GBPE_SPARSE_TRACE counts candidates and hits)
__device__ __forceinline__ void sig_bits(uint32_t pid, uint32_t& b1, uint32_t& b2, uint32_t& b3) {
    const uint32_t h = sig_hash(pid), w = (h & 31u) << 6;
    b1 = w | ((h >> 5) & 63u);
    b2 = w | ((h >> 11) & 63u);
    b3 = w | ((h >> 17) & 63u);
}
__device__ __forceinline__ bool sig_has(const uint32_t* __restrict__ sig, uint32_t pid) {
    const uint32_t h = sig_hash(pid);
    const uint64_t v = reinterpret_cast<const uint64_t*>(sig)[h & 31u];
    const uint64_t m = (1ull << ((h >> 5) & 63u)) | (1ull << ((h >> 11) & 63u)) | (1ull << ((h >> 17) & 63u));
    return (v & m) == m;
}
#endif
// global signature (k_body): no-return atomics, no test load on the merge's critical path
__device__ __forceinline__ void sig_or(uint32_t* __restrict__ sig, uint32_t pid) {
    uint32_t b1, b2, b3;
    sig_bits(pid, b1, b2, b3);
    atomicOr(&sig[b1 >> 5], 1u << (b1 & 31u));
    atomicOr(&sig[b2 >> 5], 1u << (b2 & 31u));
    atomicOr(&sig[b3 >> 5], 1u << (b3 & 31u));
}
// a sector's new signature bits gathered in LDS (body_sector's lsig)
__device__ __forceinline__ void sig_lds(uint32_t* sig, uint32_t pid) {
    uint32_t b1, b2, b3;
    sig_bits(pid, b1, b2, b3);
    atomicOr(&sig[b1 >> 5], 1u << (b1 & 31u));
    atomicOr(&sig[b2 >> 5], 1u << (b2 & 31u));
    atomicOr(&sig[b3 >> 5], 1u << (b3 & 31u));
}
// LDS signature (k_sp_bits): test first, most bits are already set
__device__ __forceinline__ void sig_set(uint32_t* __restrict__ sig, uint32_t pid) {
    uint32_t b1, b2, b3;
    sig_bits(pid, b1, b2, b3);
    const uint32_t m1 = 1u << (b1 & 31u), m2 = 1u << (b2 & 31u), m3 = 1u << (b3 & 31u);
    if (!(sig[b1 >> 5] & m1)) atomicOr(&sig[b1 >> 5], m1);
    if (!(sig[b2 >> 5] & m2)) atomicOr(&sig[b2 >> 5], m2);
    if (!(sig[b3 >> 5] & m3)) atomicOr(&sig[b3 >> 5], m3);
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
// whole-wave lane shifts (DPP wave_shr:1 / wave_shl:1, GFX9 DPP controls 0x138 /
// 0x130): lane i gets lane i-1's (i+1's) value; the lane shifted in gets 0
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}

// lsig (optional): this wave's 64-word LDS copy of the sector signature's new
// bits — a created pair sets its 3 bits there (LDS atomics), and the sector's end
// ORs each word into the global signature once (one atomic per non-zero word
// instead of three per created pair: early merges create thousands per sector)
template <typename S, int NT = LTAB_T, typename TB = Table, typename LT = LdsTab<NT>, bool LSIG = false>
__device__ __forceinline__ uint32_t body_sector(S* __restrict__ p, uint32_t* __restrict__ mp, uint32_t cnt, uint32_t a, uint32_t b,
                                uint32_t nw, LT& lt, const TB& tb, DevState* st, uint32_t* __restrict__ sig,
                                uint32_t& out_cnt, const uint32_t (&first)[5], const uint32_t (&firstm)[4],
                                uint32_t* lsig, const uint32_t* nxt, const uint32_t* nxtm BSP_ARG) {
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    const int lane = threadIdx.x & 63;
    const uint32_t pid_ab = (a << 16) | b;
    uint32_t c1 = 0, c2 = 0, out = 0, removed = 0;
    for (uint32_t c0 = 0; c0 < cnt; c0 += SP_CH) {
        BSP_CLK(q0);
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
        // neighbours across lanes without the LDS crossbar (ds_bpermute queues behind
        // the wave's and its CU's LDS atomics): DPP whole-wave shifts, readlane
        uint32_t pm1 = wave_shr1(X[5]), pm2 = wave_shr1(X[4]);
        uint32_t np = wave_shl1(X[2]);
        if (lane == 0) {
            pm1 = c1;
            pm2 = c2;
        }
        if (lane == 63) np = nx;
        X[0] = pm2;
        X[1] = pm1;
        X[6] = np;
        c1 = __builtin_amdgcn_readlane(X[5], 63);
        c2 = __builtin_amdgcn_readlane(X[4], 63);
        // h[j] = hit at the position of X[j]: a B-side (no word-start bit) after an a
        bool h[7];
        h[0] = false;
#pragma unroll
        for (int j = 1; j < 7; ++j) h[j] = X[j] == b && (X[j - 1] & TM) == a;
#ifdef GBPE_BSPROF
        const unsigned long long q1 = clock64() + (h[2] && h[3] && h[4] && h[5] && !M[0] ? 1ull : 0ull);   // (after the loads)
        BSP_ADD(0, q1 - q0);
#endif
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
                            if (LSIG) sig_lds(lsig, (nw << 16) | t2);
                            else sig_or(sig, (nw << 16) | t2);
                        }
                    } else if (h[j + 1] && tp) {
                        lds_add(lt, tb, st, (tp << 16) | nw, w);
                        if (LSIG) sig_lds(lsig, (tp << 16) | nw);
                        else sig_or(sig, (tp << 16) | nw);
                    }
                }
            }
        }
#ifdef GBPE_BSPROF
        BSP_CLK(q2);
        BSP_ADD(1, q2 - q1);
#endif
        // the wave's exclusive prefix of the kept counts from four ballots (one per
        // symbol slot) and mbcnt: no LDS round trips
        const uint32_t kc = __popc(keep);
        uint32_t excl = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t m = __ballot((keep >> k) & 1u);
            excl += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            tot += (uint32_t)__popcll(m);
        }
        const uint32_t incl = excl + kc;
        // every read of this pass happened above; writes land at or before their source
        if (nxt) {
            // the next sector's first pass (prefetched by the caller) is waited for
            // here, before this pass's stores: gfx950 counts loads and stores in one
            // vmcnt, so waiting for it at the next sector's start would drain these
            // stores too (the compiler cannot count them: vmcnt(0))
#pragma unroll
            for (int k = 0; k < 5; ++k) asm volatile("" ::"v"(nxt[k]));
#pragma unroll
            for (int k = 0; k < 4; ++k) asm volatile("" ::"v"(nxtm[k]));
        }
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
#ifdef GBPE_BSPROF
        BSP_CLK(q3);
        BSP_ADD(2, q3 - q2);
        BSP_ADD(4, 1ull);
#endif
    }
    out_cnt = out;
    BSP_CLK(q4);
    if (LSIG) {   // (SP_SIGW == 64: a word per lane; the exchange also clears it for the next sector)
        const uint32_t v = atomicExch(&lsig[lane], 0u);
        if (v) atomicOr(&sig[lane], v);
    }
    removed = wave_sum_u32(removed);   // per lane → the wave's
#ifdef GBPE_BSPROF
    BSP_ADD(3, clock64() - q4);
    BSP_ADD(5, 1ull);
#endif
    return removed;
}

// dst[i - beg] = src[i] for i in [beg, end), thread-strided, U loads in flight per
// thread: a one-load-per-trip loop waits a whole round trip per trip (the zone
// passes' window-source copies: ~3-11 trips per thread, on the zone's chain)
template <typename S, int BT, int U = 4>
__device__ __forceinline__ void copy_strided(S* __restrict__ dst, const S* __restrict__ src, uint32_t beg, uint32_t end) {
    for (uint32_t i0 = beg + threadIdx.x; i0 < end; i0 += (uint32_t)BT * U) {
        S v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + (uint32_t)u * BT;
            v[u] = i < end ? src[i] : (S)0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + (uint32_t)u * BT;
            if (i < end) dst[i - beg] = v[u];
        }
    }
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
    uint32_t tf;   // zone_one: the first thread outside the unmoved prefix
    S trash[64];   // the zone pass's unconditional stores of dropped symbols
};

__device__ __forceinline__ uint32_t lane_mask_n(uint64_t i0, uint64_t lim, int n) {
    // bits k with i0 + k < lim, k < n (n <= 32)
    const uint32_t full = n == 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    return i0 >= lim ? 0u : (i0 + n <= lim ? full : ((1u << (uint32_t)(lim - i0)) - 1u));
}

// z: the zone's length, wsrc: the stale-window source's offset in the other buffer
// (launch snapshots: no state round trip before the zone loads).
// zout: the delta table is the caller's (neither cleared nor flushed here) and m,
// the new zone length go to zout[0..1]
template <typename S, bool EXACT, int BT, int NT = LTAB_T, int ZPT_ = ZoneDim<S, BT>::ZPT, typename TB = Table>
__device__ __forceinline__ void zone_one(DevState* st, DevState* zst, uint32_t z, uint64_t wsrc, S* __restrict__ zc,
                         S* __restrict__ zo, ZoneLds<S, BT>& L,
                         LdsTab<NT>& lt, const TB& tb, uint32_t a, uint32_t b, uint32_t nw, uint32_t mc,
                         uint64_t* __restrict__ bytes, uint32_t round, uint32_t* zout = nullptr) {
    (void)round;   // phase stamps only (-DGBPE_KTRACE)
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    constexpr int ZPT = ZPT_;                // zone positions per thread (<= ZoneDim's: the LDS is sized for that)
    static_assert(ZPT <= ZoneDim<S, BT>::ZPT && ZPT * sizeof(S) % 16 == 0, "zone positions per thread");
    constexpr int V = ZPT * sizeof(S) / 16;  // 16-byte vectors per thread
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t lim = EXACT ? z : z - mc;
    const uint32_t pid_ab = (a << 16) | b;
    const uint32_t i0 = (uint32_t)t * ZPT;
    S* xs = reinterpret_cast<S*>(L.xv);
    uint32_t x[ZPT];
    uint4 v[V];
    {
        const uint4* src = reinterpret_cast<const uint4*>(zc + i0);   // zone buffers hold >= 2 tiles
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = src[k];
#pragma unroll
        for (int k = 0; k < V; ++k) L.xv[t * V + k] = v[k];
        const S* e = reinterpret_cast<const S*>(v);
#pragma unroll
        for (int k = 0; k < ZPT; ++k) x[k] = i0 + k < z ? (uint32_t)e[k] : 0u;
    }
    if (!EXACT)   // window source: global n - 2mc in the previous stream
        copy_strided<S, BT, 8>(L.wb, zo + wsrc, 0u, mc);
    if (t == 0) L.tf = BT;
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
    for (uint32_t ib = (lim > 1u ? lim : 1u) + t; ib < z; ib += 4u * BT) {   // stale tail: old pairs destroyed
        uint32_t kq[4];   // (4 pairs' reads and CASes overlap: lds_addk)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = ib + (uint32_t)k * BT;
            const uint32_t xi = i < z ? (uint32_t)xs[i] : WS, tp = i < z ? (uint32_t)xs[i - 1] & TM : 0u, ti = xi & TM;
            kq[k] = (!(xi & WS) && tp && ti && ((tp << 16) | ti) != pid_ab) ? (tp << 16) | ti : 0u;
        }
        lds_addk<4>(lt, tb, st, kq, 0xFFFFFFFFu);
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
    // The unmoved prefix: the threads before the first one holding a site, an
    // A-side or position lim - 1 keep every symbol at its own position, so they
    // store their loaded vectors straight to the other buffer (aligned) and skip
    // the LDS assembly below — late in training most merges have no site in the
    // zone at all, and the assembly is most of the zone pass's instructions.
    {
        const unsigned long long sm = __ballot((hitm | rwm) != 0u || i0 + ZPT >= lim);
        if (sm && lane == 0) atomicMin(&L.tf, (uint32_t)(wid * 64 + __ffsll((long long)sm) - 1));
    }
    // block exclusive scan of the kept counts; tail survivors sum to m
    const uint32_t kc = __popc(keep);
    const uint32_t incl = wave_scan_incl_u32(kc), tl = wave_sum_u32(__popc(surv & ~below));
    if (lane == 63) L.wsum[wid] = incl;
    if (lane == 0) L.wtail[wid] = tl;
    __syncthreads();
    if (t == 0) KT(7);
    const uint32_t tf = L.tf, F = tf * ZPT;
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
    if ((uint32_t)t < tf) {
        uint4* dz = reinterpret_cast<uint4*>(zo + i0);
#pragma unroll
        for (int k = 0; k < V; ++k) dz[k] = v[k];
        if ((uint32_t)t + 1u == tf) xs[swz(F - 1u)] = (S)x[ZPT - 1];   // the window's left neighbour may be it
    } else if (keep | rwm) {
        uint32_t wsm = 0;
#pragma unroll
        for (int k = 0; k < ZPT; ++k) {
            const bool rw = (rwm >> k) & 1u;
            const uint32_t y = rw ? (nw | (x[k] & WS)) : x[k];
            wsm |= ((x[k] & WS) ? 1u : 0u) << k;
            const uint32_t o = pre + (uint32_t)__popc(keep & ((1u << k) - 1u));
            S* dst = ((keep >> k) & 1u) ? &xs[swz(o)] : &L.trash[lane];
            *dst = (S)y;
        }
        for (uint32_t r = rwm; r; r &= r - 1) {
            const int k = __ffs(r) - 1;
            zc[i0 + k] = (S)(nw | (((wsm >> k) & 1u) ? WS : 0u));
        }
    }
    if (t == 0) KT(8);
    if (!EXACT && m) {
        __syncthreads();
        const uint32_t woff = mc - m;
        for (uint32_t jb = t; jb < m; jb += 4u * BT) {
            uint32_t kq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = jb + (uint32_t)k * BT;
                kq[k] = 0u;
                if (j < m) {
                    const uint32_t x1 = L.wb[woff + j];
                    // left of the window: the last kept survivor (Kz > 0: the zone holds >= 5 mc)
                    const uint32_t x0 = j ? (uint32_t)L.wb[woff + j - 1] : (Kz ? (uint32_t)xs[swz(Kz - 1)] : 0u);
                    xs[swz(Kz + j)] = (S)x1;
                    if (!(x1 & WS) && (x0 & TM) && (x1 & TM)) kq[k] = ((x0 & TM) << 16) | (x1 & TM);
                }
            }
            lds_addk<4>(lt, tb, st, kq, 1u);
        }
    }
    __syncthreads();
    if (t == 0) KT(9);
    {
        const uint32_t tot = Kz + m, nfull = tot / PV;
        uint4* dst = reinterpret_cast<uint4*>(zo);
        for (uint32_t q = F / PV + t; q < nfull; q += BT) dst[q] = L.xv[q ^ ((q >> 3) & 7u)];
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
__device__ __forceinline__ void zone_seg(DevState* st, DevState* zst, const DevState& gs, const DevState& zs, S* __restrict__ zc,
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
    const uint64_t src0 = win_src0(gs, mc);
    if (!EXACT && q0 < q1)   // L.wb[j] = source[f + j], f = q0 - 1 (or 0)
        copy_strided<S, BT>(L.wb, zo + src0, q0 ? q0 - 1u : 0u, q1);
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
    const uint32_t incl = wave_scan_incl_u32(kc), tl = wave_sum_u32(__popc(surv & ~below));
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
        sp = wave_sum_u32(sp);
        sk = wave_sum_u32(sk);
        stt = wave_sum_u32(stt);
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
struct SelShard {
    uint32_t zf = 3;         // zone rule: z >= max(2 mc + mc_prev, zf mc) + 2 (trainer zone_f)
    uint32_t sub = 1;        // k_body workgroups per bitmap word (1, 2, 4: a row of few words, body_grid)
    uint32_t k2 = 0;         // paired launches allowed (the zone_one form: zone_two)
};

// The second merge of a paired launch.  With P1 > P2 the table's two
// largest keys and P2's tokens disjoint from P1's, merging P1 leaves P2's count as
// it is and every pair it creates is bounded by a pair other than P1 and P2 that
// loses to P2 (on equal counts too: the new id is larger than every token), so P2
// is the argmax after P1 — up to the stale window the reference compaction adds,
// which zone_two checks before the second merge runs (ref mode).
struct Sel2 {
    uint32_t a = 0, b = 0, mc = 0;
    bool dbl = false;        // candidate (zone_two decides in ref mode; exact mode always runs it)
};

template <int BT, bool TOP2>
__device__ __forceinline__ bool sel_inline(DevState* st, DevState* zst, const uint64_t* __restrict__ part, uint32_t npart,
                           bool exact, bool zone1, const Table& tb, uint32_t* __restrict__ log,
                           uint32_t* __restrict__ grpsum, uint32_t& a, uint32_t& b, uint32_t& nw, uint32_t& mc,
                           uint32_t& md, Sel2& s2, const DevState*& gsnap, const DevState*& zsnap,
                           const SelShard sh = SelShard(), bool commit = true) {
    __shared__ uint64_t s_red[BT / 64], s_red2[BT / 64];
    constexpr int NW = sizeof(DevState) / 4;
    __shared__ union {
        DevState d;
        uint32_t w[NW];
    } s_g, s_z;
    const int t = threadIdx.x;
    // the partial maxima (two keys per k_refresh workgroup, one 16-byte load) and
    // snapshots of both states load together (one round trip, not one per field)
    if (t < NW) s_g.w[t] = reinterpret_cast<const uint32_t*>(st)[t];
    else if (zst && t < 2 * NW) s_z.w[t - NW] = reinterpret_cast<const uint32_t*>(zst)[t - NW];
    uint64_t best = 0, second = 0;   // (TOP2: only the paired form reduces a second key)
    for (uint32_t i = t; i < npart; i += BT) {
        if constexpr (TOP2) {
            const ulonglong2 v = reinterpret_cast<const ulonglong2*>(part)[i];
            top2_merge(best, second, v.x, v.y);
        } else {
            const uint64_t v = part[2 * i];
            best = v > best ? v : best;
        }
    }
    __syncthreads();
    const DevState& g = s_g.d;
    gsnap = &s_g.d;
    zsnap = &s_z.d;
    md = g.merges_done;   // the merge index (a paired launch runs two: launches and merges part ways)
    if (!(md < g.budget && !g.stop && !g.sp_abort)) return false;
    if constexpr (TOP2) {
        wave_top2_u64(best, second, best, second);
        if ((t & 63) == 0) {
            s_red[t >> 6] = best;
            s_red2[t >> 6] = second;
        }
        __syncthreads();
        best = s_red[0];
        second = s_red2[0];
#pragma unroll
        for (int w = 1; w < BT / 64; ++w) top2_merge(best, second, s_red[w], s_red2[w]);
    } else {
        best = wave_max_u64(best);
        if ((t & 63) == 0) s_red[t >> 6] = best;
        __syncthreads();
        best = s_red[0];
#pragma unroll
        for (int w = 1; w < BT / 64; ++w) best = s_red[w] > best ? s_red[w] : best;
    }
    mc = (uint32_t)(best >> 32);
    const uint32_t pid = ~(uint32_t)best;
    a = pid >> 16;
    b = pid & 0xFFFFu;
    nw = g.next_id;
    const bool stop = mc < 2u || nw > 0xFFFFu;                                          // train.wgsl:345-348
    const bool bad = !stop && !exact && g.is_last && (uint64_t)(uint32_t)(g.n - g.Bp) < 2ull * mc;   // cannot happen
    // zone misfit: this merge's window source must lie in the zone's stale buffer
    // (n - 2mc >= Bp, where n - Bp >= z - mc_prev: the last merge removed <= mc_prev
    // body symbols), and the zone keeps >= zf mc for the merges after it
    const uint32_t mc_prev = g.mc_prev;
    const uint64_t zneed = std::max<uint64_t>(2ull * mc + mc_prev, (uint64_t)sh.zf * mc) + 2u;
    const bool abort = !stop && !bad && !exact && (uint64_t)g.zlast < zneed;
    const bool go = !stop && !bad && !abort;
    {   // the second merge: P2 disjoint from P1, its own stop rules, and the zone rule on the
        // zone the first leaves (>= z - mc) with mc as its mc_prev
        const uint32_t mc2 = (uint32_t)(second >> 32), pid2 = ~(uint32_t)second;
        const uint32_t a2 = pid2 >> 16, b2 = pid2 & 0xFFFFu;
        const uint64_t zneed2 = (uint64_t)mc + std::max<uint64_t>(2ull * mc2 + mc, (uint64_t)sh.zf * mc2) + 2u;
        s2.a = a2;
        s2.b = b2;
        s2.mc = mc2;
        s2.dbl = sh.k2 && zone1 && go && md + 2u <= g.budget && mc2 >= 2u && nw + 1u <= 0xFFFFu && a2 != a &&
                 a2 != b && b2 != a && b2 != b && (exact || (uint64_t)g.zlast >= zneed2);
    }
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
            } else {
                const uint32_t idx = table_find(tb, pid);
                if (idx == 0xFFFFFFFFu) {
                    atomicOr(&st->err, ERR_PAIR_MISSING);
                } else {
                    // every (a,b) occurrence is a merge site: count -= mc, atomically, since
                    // other workgroups may already add this merge's stale-window pairs
                    atomicSub(&tb.slots[idx].y, mc);
                    tb.dirty[idx >> BLK_LOG2] = 1u;
                }
                log[md * 4 + 0] = a;
                log[md * 4 + 1] = b;
                log[md * 4 + 2] = nw;
                log[md * 4 + 3] = mc;
                if (s2.dbl) {   // (k_refresh keeps it only if the zone workgroup accepts it)
                    log[md * 4 + 4] = s2.a;
                    log[md * 4 + 5] = s2.b;
                    log[md * 4 + 6] = nw + 1u;
                    log[md * 4 + 7] = s2.mc;
                    st->mc2 = s2.mc;
                }
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
                zst->merges_done = md + 1u;
                st->sel_round = md + 1u;
            }
        }
        if (go) {   // group sums of a multi-tile zone pass start at zero
            const uint32_t ngrp = (uint32_t)gbpe_div_up(gbpe_div_up(s_z.d.n, TILE), GRP);
            for (uint32_t q = t; q < ngrp; q += BT) grpsum[q * GSTR] = 0u;
        }
    }
    return go;
}

// the paired launch's verdict word (ZSegState pad[1], never zeroed): the launch's
// epoch << 2 | 2 (decided) | 1 (accepted)
__device__ __forceinline__ uint32_t* pair_word(ZSegState* zg) { return &zg->pad[1]; }

// Zone workgroup of a paired launch: both merges in one pass over the
// zone — one load, the first merge's zone assembled in LDS, the verdict, the second
// merge on that LDS copy, one store of each zone buffer and one flush.
//  * As in zone_one, the threads before the first one holding a site, an A-side or
//    position lim - 1 keep their symbols in place (the unmoved prefix, rounded down
//    to whole 128-byte swizzle groups): they neither assemble in LDS nor reload,
//    and LDS holds that prefix unswizzled (at1 / at2 read either layout).
//  * The second merge's stale window comes from the first merge's current buffer
//    with the first's A-side rewrites in place (the reference's ping-pong): those
//    symbols, [z - mc - 2 mc2, + mc2) of the loaded zone, are staged in wb2 with the
//    rewrites applied before LDS is overwritten.
//  * Ref-mode verdict: the first merge's stale window (and the tail it replaces) may
//    lift a pair over P2 or change P2's count.  Every zone delta of merge 1 is in
//    the table (an overflow rejects): P2's net delta must be 0, and every window
//    pair with a positive net delta must stay below P2 with its count read now (the
//    body workgroups' adds to a pair without nw are decrements, so the read bounds
//    the final count from above).  Pairs of nw come from sites (bounded, Sel2)
//    except the window's first pair, whose left symbol (the last kept survivor at
//    lim - 1) is checked: nw or not kept there rejects.  The window pairs' counts
//    are loaded before the first merge's assembly, so the round trip overlaps it.
//  * zo ends as the first merge's output with the second's A-side rewrites (a later
//    window reads it), zc as the second's output.  Rejected: the first merge's
//    output goes to zo and its rewrites to zc, as zone_one leaves them.
template <typename S, bool EXACT, int BT, int NT, int ZPT>
__device__ __forceinline__ void zone_two(DevState* st, DevState* zst, const DevState& gs, uint32_t z, S* __restrict__ zc,
                                         S* __restrict__ zo, ZSegState* zg, ZoneLds<S, BT>& L, S* __restrict__ wb2,
                                         LdsTab<NT>& ltab, const Table& tb, uint32_t a, uint32_t b, uint32_t nw,
                                         uint32_t mc, const Sel2& s2, uint64_t* __restrict__ bytes, uint32_t round) {
    (void)round;   // phase stamps only (-DGBPE_KTRACE: 2 loaded, 3 merge-1 deltas, 7 merge 1 in LDS, 8 verdict,
                   // 9 merge 2 in LDS, 4 stored; the caller stamps 5 after the flush)
    constexpr uint32_t WS = Sym<S>::WS, TM = Sym<S>::TM;
    static_assert(ZPT == ZoneDim<S, BT>::ZPT && ZPT * sizeof(S) % 16 == 0, "zone positions per thread");
    constexpr int V = ZPT * sizeof(S) / 16;
    constexpr uint32_t PV = 16 / sizeof(S), PVL = sizeof(S) == 2 ? 3 : 2;
    constexpr uint32_t TG = ZPT * sizeof(S) >= 128 ? 1u : 128u / (ZPT * sizeof(S));   // threads per swizzle group
    constexpr int KV = (ZoneDim<S, BT>::ZWIN + BT - 1) / BT;   // window pairs per thread (m <= mc <= ZWIN)
    auto swz = [](uint32_t o) -> uint32_t {   // 16-byte chunks XOR-swizzled in groups of 8 (zone_one)
        const uint32_t c = o >> PVL;
        return ((c ^ ((c >> 3) & 7u)) << PVL) | (o & (PV - 1u));
    };
    __shared__ uint32_t s_rej, s_x0, s_tf1, s_tf2;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint32_t a2 = s2.a, b2 = s2.b, n2 = nw + 1u, mc2 = s2.mc;
    const uint32_t pid1 = (a << 16) | b, pid2 = (a2 << 16) | b2;
    // both merges' tails and windows are <= 2 (mc + mc2) pairs: a table at <= ~1/2 load
    uint32_t nslot = 1024u;
    while (nslot < (uint32_t)NT && nslot < 4u * (mc + mc2)) nslot <<= 1;
    LdsView lt = lds_view(ltab, nslot);
    lds_clear(lt);
    if (t == 0) {
        s_rej = 0u;
        s_x0 = 0u;
        s_tf1 = BT;
        s_tf2 = BT;
    }
    // P2's home slot for its commit, loaded while merge 1 runs
    const uint32_t h2i = gbpe_fmix32(pid2) & tb.mask;
    uint64_t h2 = 0;
    if (t == 0)
        h2 = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&tb.slots[h2i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    if (!EXACT) copy_strided<S, BT, 8>(L.wb, zo + win_src0(gs, mc), 0u, mc);
    __syncthreads();
    if (t == 0) KT(2);
    KTW(0);
    // ── merge 1: zone_one's site masks and deltas ──
    const uint32_t lim = EXACT ? z : z - mc;
    uint32_t rwm = 0, wsm = 0, keep = 0;
    {
        const uint32_t xm2 = i0 >= 2 ? (uint32_t)xs[i0 - 2] : 0u, xm1 = i0 >= 1 ? (uint32_t)xs[i0 - 1] : 0u;
        const uint32_t nxr = i0 + ZPT < z ? (uint32_t)xs[i0 + ZPT] : 0u;
        uint32_t eb = 0, ea = 0;
#pragma unroll
        for (int k = 0; k < ZPT; ++k) {
            eb |= (x[k] == b ? 1u : 0u) << k;
            ea |= ((x[k] & TM) == a ? 1u : 0u) << k;
            wsm |= ((x[k] & WS) ? 1u : 0u) << k;
        }
        const uint32_t inb = lane_mask_n(i0, z, ZPT);
        const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a ? 1u : 0u)) & inb;
        const uint32_t h_m1 = (i0 >= 1 && i0 - 1 < z && xm1 == b && (xm2 & TM) == a) ? 1u : 0u;
        const uint32_t h_32 = (nxr == b && (ea >> (ZPT - 1))) ? 1u : 0u;
        const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_32 << (ZPT + 1));
        const uint32_t below = lane_mask_n(i0, lim, ZPT);
        const uint32_t surv = inb & ~hitm;
        keep = surv & below;
        rwm = ((hitm >> 1) | (h_32 << (ZPT - 1))) & inb;
        uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
        if (t == 0) KT(10);
        KTW(1);
        for (uint32_t ib = (lim > 1u ? lim : 1u) + t; ib < z; ib += 4u * BT) {   // stale tail: old pairs destroyed
            uint32_t kq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t i = ib + (uint32_t)k * BT;
                const uint32_t xi = i < z ? (uint32_t)xs[i] : WS, tp = i < z ? (uint32_t)xs[i - 1] & TM : 0u, ti = xi & TM;
                kq[k] = (!(xi & WS) && tp && ti && ((tp << 16) | ti) != pid1) ? (tp << 16) | ti : 0u;
            }
            lds_addk<4>(lt, tb, st, kq, 0xFFFFFFFFu);
        }
        if (t == 0) KT(11);
        KTW(2);
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
            if (tp && ti && ((tp << 16) | ti) != pid1) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
            if (!h0) {
                if (hm) {
                    const uint32_t t2 = hp ? nw : ti;
                    if (t2) lds_add(lt, tb, st, (nw << 16) | t2, 1u);
                } else if (hp && tp) {
                    lds_add(lt, tb, st, (tp << 16) | nw, 1u);
                }
            }
        }
        KTW(3);
        if (!EXACT) {
            // the second merge's window source [w2, w2 + mc2) (w2 >= 0: sel_inline's rule), strided over
            // every thread; an A-side (a followed by a B-side b, train.wgsl:482-488) reads back as nw
            const uint32_t w2 = z - mc - 2u * mc2;
            for (uint32_t p = w2 + t; p < w2 + mc2; p += BT) {
                const uint32_t xp = xs[p], xn = p + 1u < z ? (uint32_t)xs[p + 1u] : 0u;
                wb2[p - w2] = (S)(((xp & TM) == a && xn == b) ? (nw | (xp & WS)) : xp);
            }
            if (lim >= 1u && lim - 1u >= i0 && lim - 1u < i0 + ZPT) {   // the window's left neighbour, if kept
                const uint32_t k = lim - 1u - i0;
                if ((keep >> k) & 1u)
                    s_x0 = 0x80000000u | (((rwm >> k) & 1u) ? (nw | (x[k] & WS)) : x[k]);
            }
        }
        KTW(4);
        {   // the unmoved prefix (zone_one)
            const unsigned long long sm = __ballot((hitm | rwm) != 0u || i0 + ZPT >= lim);
            if (sm && lane == 0) atomicMin(&s_tf1, (uint32_t)(wid * 64 + __ffsll((long long)sm) - 1));
        }
        const uint32_t kc = __popc(keep);
        const uint32_t incl = wave_scan_incl_u32(kc), tl = wave_sum_u32(__popc(surv & ~below));
        if (lane == 63) L.wsum[wid] = incl;
        if (lane == 0) L.wtail[wid] = tl;
        KTW(5);
    }
    __syncthreads();
    if (t == 0) KT(3);
    uint32_t Kz = 0, m = 0, pre = 0;
    {
        uint32_t incl_w = 0;
#pragma unroll
        for (int w2 = 0; w2 < BT / 64; ++w2) {
            incl_w += w2 < wid ? L.wsum[w2] : 0u;
            Kz += L.wsum[w2];
            m += L.wtail[w2];
        }
        pre = incl_w + wave_scan_incl_u32(__popc(keep)) - __popc(keep);
    }
    const uint32_t tf1 = s_tf1 / TG * TG, F1 = tf1 * ZPT;
    auto at1 = [&](uint32_t p) -> uint32_t {   // the first merge's zone in LDS (position p < z1)
        return p < F1 ? (uint32_t)xs[p] : (uint32_t)xs[swz(p)];
    };
    // the verdict's window pairs: their counts load now and arrive during the assembly
    const uint32_t woff = mc - m;
    uint32_t vq[KV];
    uint64_t vh[KV];
    if (!EXACT) {
        const uint32_t x0 = s_x0;
        if (t == 0 && m && Kz && !(x0 >> 31)) s_rej = 1u;   // the last kept survivor is not at lim - 1
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const uint32_t j = (uint32_t)t + (uint32_t)k * BT;
            vq[k] = 0u;
            vh[k] = 0;
            if (j < m) {
                const uint32_t x1 = L.wb[woff + j];
                const uint32_t xl = j ? (uint32_t)L.wb[woff + j - 1] : (Kz ? (x0 & 0x7FFFFFFFu) : 0u);
                if (!(x1 & WS) && (xl & TM) && (x1 & TM)) {
                    const uint32_t q = ((xl & TM) << 16) | (x1 & TM);
                    if ((q >> 16) == nw) s_rej = 1u;   // a pair of the new token that no site made
                    else vq[k] = q;
                }
                // (P1's count is 0 after its commit; P2: its net delta.)  Plain loads, not waited for
                // here: a line older than the body workgroups' adds to this pair holds a count at
                // least its final one (those adds are decrements), which only makes the check stricter
                if (vq[k] && vq[k] != pid1 && vq[k] != pid2)
                    vh[k] = reinterpret_cast<const uint64_t*>(tb.slots)[gbpe_fmix32(vq[k]) & tb.mask];
            }
        }
    }
    KTW(6);
    // the first merge's zone in LDS past the unmoved prefix (every read of the old copy is done)
    if ((uint32_t)t >= tf1) {   // (8-symbol chunks no lane of the wave keeps are skipped: the stale tail)
#pragma unroll
        for (int c8 = 0; c8 < ZPT; c8 += 8) {
            if (!__any((keep >> c8) & 0xFFu)) continue;
#pragma unroll
            for (int k = c8; k < c8 + 8; ++k) {
                const uint32_t y = ((rwm >> k) & 1u) ? (nw | (x[k] & WS)) : x[k];
                const uint32_t o = pre + (uint32_t)__popc(keep & ((1u << k) - 1u));
                S* dst = ((keep >> k) & 1u) ? &xs[swz(o)] : &L.trash[lane];
                *dst = (S)y;
            }
        }
    }
    KTW(7);
    if (!EXACT && m) {
        __syncthreads();
        KTW(8);
        for (uint32_t jb = t; jb < m; jb += 4u * BT) {
            uint32_t kq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = jb + (uint32_t)k * BT;
                kq[k] = 0u;
                if (j < m) {
                    const uint32_t x1 = L.wb[woff + j];
                    const uint32_t x0 = j ? (uint32_t)L.wb[woff + j - 1] : (Kz ? at1(Kz - 1) : 0u);
                    xs[swz(Kz + j)] = (S)x1;
                    if (!(x1 & WS) && (x0 & TM) && (x1 & TM)) kq[k] = ((x0 & TM) << 16) | (x1 & TM);
                }
            }
            lds_addk<4>(lt, tb, st, kq, 1u);
        }
    }
    KTW(9);
    __syncthreads();
    const uint32_t z1 = Kz + m;
    if (t == 0) KT(7);
    // ── the verdict ──
    bool rej = false;
    if (!EXACT) {
        if (t == 0) rej = s_rej != 0u || *lt.ovf != 0u || lds_find(lt, pid2) != 0u;
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            if (!vq[k] || vq[k] == pid2) continue;
            const uint32_t d = lds_find(lt, vq[k]);
            if ((int32_t)d <= 0) continue;
            uint32_t cnt = 0;
            if (vq[k] != pid1) {
                if ((uint32_t)vh[k] == vq[k]) {
                    cnt = (uint32_t)(vh[k] >> 32);
                } else {
                    const uint32_t idx = table_find(tb, vq[k]);
                    cnt = idx == 0xFFFFFFFFu ? 0u : __hip_atomic_load(&tb.slots[idx].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if ((int32_t)cnt < 0) cnt = 0;
            }
            const uint64_t c2 = (uint64_t)cnt + d;
            if (c2 > mc2 || (c2 == mc2 && vq[k] < pid2)) rej = true;
        }
        rej = __syncthreads_or(rej) != 0;
    }
    if (t == 0) {
        st->pair_cand += 1u;   // (diagnostics: one zone workgroup per launch)
        if (rej) st->pair_rej += 1u;
        if (!rej) {   // commit P2: every occurrence is a site of the second merge
            const uint32_t idx = (uint32_t)h2 == pid2 ? h2i : table_find(tb, pid2);
            if (idx == 0xFFFFFFFFu) {
                atomicOr(&st->err, ERR_PAIR_MISSING);
            } else {
                atomicSub(&tb.slots[idx].y, mc2);
                tb.dirty[idx >> BLK_LOG2] = 1u;
            }
            st->acc2 = 1u;
        }
        __hip_atomic_store(pair_word(zg), (gs.epoch << 2) | (rej ? 2u : 3u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        KT(8);
    }
    // the LDS zone's swizzled part [from, tot) to dst as 16-byte vectors (from: a swizzle-group boundary)
    auto store_lds = [&](S* dst, uint32_t from, uint32_t tot) {
        const uint32_t nfull = tot / PV;
        uint4* dv = reinterpret_cast<uint4*>(dst);
        for (uint32_t qv = from / PV + t; qv < nfull; qv += BT) dv[qv] = L.xv[qv ^ ((qv >> 3) & 7u)];
        for (uint32_t j = std::max(nfull * PV, from) + t; j < tot; j += BT) dst[j] = xs[swz(j)];
    };
    auto store_regs = [&](S* dst, const uint32_t (&y)[ZPT]) {   // this thread's ZPT symbols as vectors
        S e[ZPT];
#pragma unroll
        for (int k = 0; k < ZPT; ++k) e[k] = (S)y[k];
        uint4* dv = reinterpret_cast<uint4*>(dst + i0);
#pragma unroll
        for (int k = 0; k < V; ++k) dv[k] = reinterpret_cast<const uint4*>(e)[k];
    };
    if (rej) {   // merge 1 alone: its zone to zo, its rewrites in place in zc (zone_one's result)
        for (uint32_t r = rwm; r; r &= r - 1) {
            const int k = __ffs(r) - 1;
            zc[i0 + k] = (S)(nw | (((wsm >> k) & 1u) ? WS : 0u));
        }
        if ((uint32_t)t < tf1) store_regs(zo, x);
        store_lds(zo, F1, z1);
        lds_flush<NT / BT>(lt, tb, st);
        if (t == 0) {
            zst->m = m;
            zst->valid_total = z1 + 1u;
            atomicAdd(bytes, (uint64_t)sizeof(S) * ((uint64_t)z + (EXACT ? 0u : mc) + z1));
        }
        return;
    }
    // ── merge 2 on the first merge's zone (registers for the prefix, LDS past it) ──
    uint32_t Kz2 = 0, m2 = 0, F2 = 0;
    {
        const uint32_t lim2 = EXACT ? z1 : z1 - mc2;
        auto X = [&](uint32_t p) -> uint32_t { return p < z1 ? at1(p) : 0u; };
        if ((uint32_t)t >= tf1) {   // (the prefix threads' symbols are their own, unchanged)
#pragma unroll
            for (int k = 0; k < ZPT; ++k) x[k] = X(i0 + k);
        }
        const uint32_t xm2 = i0 >= 2 ? X(i0 - 2) : 0u, xm1 = i0 >= 1 ? X(i0 - 1) : 0u, nxr = X(i0 + ZPT);
        uint32_t eb = 0, ea = 0, wsm2 = 0;
#pragma unroll
        for (int k = 0; k < ZPT; ++k) {
            eb |= (x[k] == b2 ? 1u : 0u) << k;
            ea |= ((x[k] & TM) == a2 ? 1u : 0u) << k;
            wsm2 |= ((x[k] & WS) ? 1u : 0u) << k;
        }
        const uint32_t inb = lane_mask_n(i0, z1, ZPT);
        const uint32_t hitm = eb & ((ea << 1) | ((xm1 & TM) == a2 ? 1u : 0u)) & inb;
        const uint32_t h_m1 = (i0 >= 1 && i0 - 1 < z1 && xm1 == b2 && (xm2 & TM) == a2) ? 1u : 0u;
        const uint32_t h_32 = (nxr == b2 && (ea >> (ZPT - 1))) ? 1u : 0u;
        const uint64_t hbits = (uint64_t)h_m1 | ((uint64_t)hitm << 1) | ((uint64_t)h_32 << (ZPT + 1));
        const uint32_t below = lane_mask_n(i0, lim2, ZPT);
        const uint32_t surv = inb & ~hitm, keep2 = surv & below;
        const uint32_t rw2 = ((hitm >> 1) | (h_32 << (ZPT - 1))) & inb;
        uint32_t rel = ((uint32_t)hbits | (uint32_t)(hbits >> 1) | (uint32_t)(hbits >> 2)) & below & inb;
        for (uint32_t ib = (lim2 > 1u ? lim2 : 1u) + t; ib < z1; ib += 4u * BT) {   // stale tail: old pairs destroyed
            uint32_t kq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t i = ib + (uint32_t)k * BT;
                const uint32_t xi = i < z1 ? X(i) : WS, tp = i < z1 ? X(i - 1) & TM : 0u, ti = xi & TM;
                kq[k] = (!(xi & WS) && tp && ti && ((tp << 16) | ti) != pid2) ? (tp << 16) | ti : 0u;
            }
            lds_addk<4>(lt, tb, st, kq, 0xFFFFFFFFu);
        }
        while (rel) {
            const int k = __ffs(rel) - 1;
            rel &= rel - 1;
            const uint32_t i = i0 + k;
            if (i == 0) continue;
            const uint32_t xi = x[k];
            if (xi & WS) continue;
            const uint32_t xp = X(i - 1);
            const bool hm = (hbits >> k) & 1u, h0 = (hbits >> (k + 1)) & 1u, hp = (hbits >> (k + 2)) & 1u;
            const uint32_t tp = xp & TM, ti = xi & TM;
            if (tp && ti && ((tp << 16) | ti) != pid2) lds_add(lt, tb, st, (tp << 16) | ti, 0xFFFFFFFFu);
            if (!h0) {
                if (hm) {
                    const uint32_t t2 = hp ? n2 : ti;
                    if (t2) lds_add(lt, tb, st, (n2 << 16) | t2, 1u);
                } else if (hp && tp) {
                    lds_add(lt, tb, st, (tp << 16) | n2, 1u);
                }
            }
        }
        // the first merge's zone with the second's A-side rewrites -> zo (a later window reads it)
        uint32_t y[ZPT];
#pragma unroll
        for (int k = 0; k < ZPT; ++k) y[k] = ((rw2 >> k) & 1u) ? (n2 | (x[k] & WS)) : x[k];
        if (i0 < z1) store_regs(zo, y);
        {
            const unsigned long long sm = __ballot((hitm | rw2) != 0u || i0 + ZPT >= lim2);
            if (sm && lane == 0) atomicMin(&s_tf2, (uint32_t)(wid * 64 + __ffsll((long long)sm) - 1));
        }
        const uint32_t kc = __popc(keep2);
        const uint32_t incl = wave_scan_incl_u32(kc), tl = wave_sum_u32(__popc(surv & ~below));
        if (lane == 63) L.wsum[wid] = incl;
        if (lane == 0) L.wtail[wid] = tl;
        __syncthreads();   // (every read of the first merge's LDS zone is done)
        uint32_t pre2 = incl - kc;
#pragma unroll
        for (int w2 = 0; w2 < BT / 64; ++w2) {
            pre2 += w2 < wid ? L.wsum[w2] : 0u;
            Kz2 += L.wsum[w2];
            m2 += L.wtail[w2];
        }
        const uint32_t tf2 = s_tf2 / TG * TG;
        F2 = tf2 * ZPT;
        if ((uint32_t)t < tf2) {   // the unmoved prefix: its symbols are the second merge's output too
            store_regs(zc, y);
        } else {
#pragma unroll
            for (int c8 = 0; c8 < ZPT; c8 += 8) {
                if (!__any((keep2 >> c8) & 0xFFu)) continue;
#pragma unroll
                for (int k = c8; k < c8 + 8; ++k) {
                    const uint32_t o = pre2 + (uint32_t)__popc(keep2 & ((1u << k) - 1u));
                    S* dst = ((keep2 >> k) & 1u) ? &xs[swz(o)] : &L.trash[lane];
                    *dst = (S)y[k];
                }
            }
        }
        if (!EXACT && m2) {
            __syncthreads();
            const uint32_t woff2 = mc2 - m2;
            // left of the window: the last kept survivor, in the second layout past F2, else the first's
            const uint32_t xk = Kz2 ? (Kz2 - 1u >= F2 ? (uint32_t)xs[swz(Kz2 - 1u)] : at1(Kz2 - 1u)) : 0u;
            for (uint32_t jb = t; jb < m2; jb += 4u * BT) {
                uint32_t kq[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t j = jb + (uint32_t)k * BT;
                    kq[k] = 0u;
                    if (j < m2) {
                        const uint32_t x1 = wb2[woff2 + j];
                        const uint32_t x0 = j ? (uint32_t)wb2[woff2 + j - 1] : xk;
                        xs[swz(Kz2 + j)] = (S)x1;
                        if (!(x1 & WS) && (x0 & TM) && (x1 & TM)) kq[k] = ((x0 & TM) << 16) | (x1 & TM);
                    }
                }
                lds_addk<4>(lt, tb, st, kq, 1u);
            }
        }
        __syncthreads();
    }
    const uint32_t z2 = Kz2 + m2;
    if (t == 0) KT(9);
    store_lds(zc, F2, z2);
    if (t == 0) KT(4);
    lds_flush<NT / BT>(lt, tb, st);
    if (t == 0) {
        zst->m = m + m2;
        zst->valid_total = z2 + 1u;   // survivors + 1 (k_refresh checks it against the new layout)
        atomicAdd(bytes, (uint64_t)sizeof(S) * ((uint64_t)z + (EXACT ? 0u : mc) + z1 + z2));
    }
}

// Body pass: blocks [0, nbody) each own `wpg` consecutive bitmap words of
// (a-row & b-row), tested PW words at a time: the candidate sectors whose pair
// signature may hold (a, b) are merged (one wave per sector).  At most one
// workgroup per CU (a larger grid's selection repeats and scheduling rounds cost
// more than the bitmap words), and as many as the row has words up to that: a
// word's candidates are then merged by one workgroup's waves in parallel, not
// queued behind other words' (body_grid).  Blocks >= nbody copy the stale-window
// source [n - 2mc - Bp, + mc) of the zone's other buffer to `wtmp`.
// With `zst` (zone <= ZMAX), block nbody runs the whole zone pass (zone_one) and
// there are no copy blocks: one launch merges body and zone.
// A paired launch (the 256-thread form, Sel2) tests each bitmap word for both
// merges, merges the first's candidate sectors, then — once the zone workgroup
// accepted the second (ref mode) — the second's.  A sector is owned by one
// workgroup for both, so its two merges run in order.
#ifdef GBPE_ZP_OFF
constexpr bool ZP_OFF = true;
#else
constexpr bool ZP_OFF = false;
#endif
constexpr uint32_t SP_PW = 64;               // bitmap words tested per pass (one per lane of wave 0)
constexpr uint32_t SP_CAP = SP_PW * 32;      // candidate sectors per pass
template <uint32_t CAP>
struct BodyCandT {
    uint32_t sec[CAP];
    uint2 ext[CAP];
};
using BodyCand = BodyCandT<SP_CAP>;
// the zone workgroup's LDS (+ in the paired form its own delta table: merge 1's
// stale tail and window are ~2 mc distinct pairs, up to ~3.3K at the form's largest
// zones, which the 1,024-slot table shared with the body overflowed into global adds)
// (u32 zones: 2,048 slots, so two workgroups still fit a CU's LDS — the paired form's
// grid is the CU count + 1)
template <typename S> constexpr int zp_lt() { return sizeof(S) == 2 ? 4096 : 2048; }
template <typename S, int BT, int ZLT>
struct ZoneWg {
    ZoneLds<S, BT> z;
    LdsTab<ZLT> lt;
    S wb2[ZLT > 1 ? ZoneDim<S, BT>::ZWIN : 1];   // zone_two: the second merge's window source
};
template <typename S, int BT, int ZLT = 1>
union BodyLds {   // body workgroups use the candidate arrays, the zone workgroup the zone
    ZoneWg<S, BT, ZLT> zw;
    BodyCandT<(ZLT > 1 ? 2u : 1u) * SP_CAP> c;   // the paired form: both merges' lists
};

// ZSEG: the form for zones of 32K-1M symbols: blocks [0, zone1) run the zone
// segments (zone_seg) beside the body blocks, and zone_one is not compiled in
// (with both, every form spilled to scratch)
// zb0 / zb1: the zone buffers by the step's parity (zb0 holds the zone at merge 0
// of the step); a merge of odd index finds it in zb1
template <typename S, bool EXACT, int BT, int ZPT = ZoneDim<S, BT>::ZPT, bool ZSEG = false>
__global__ __launch_bounds__(BT) void k_body(DevState* st, uint32_t round, S* __restrict__ body, uint2* __restrict__ sec,
                                              uint32_t* __restrict__ bits, uint32_t W, uint32_t wpg,
                                              uint32_t* __restrict__ sig, Table tb, uint32_t nbody,
                                              S* __restrict__ zb1, S* __restrict__ wtmp,
                                              uint32_t clog, DevState* zst, S* __restrict__ zb0, uint32_t zone1,
                                              const uint64_t* __restrict__ part, uint32_t npart, uint32_t* __restrict__ log,
                                              uint32_t* __restrict__ grpsum, uint64_t* __restrict__ wg_bytes,
                                              Table dtb, SelShard sh, uint32_t* __restrict__ lmul,
                                              ZSegState* __restrict__ zg = nullptr) {
    constexpr int KB_LT = ZSEG ? 4096 : LTAB_T;   // (4096 for every 1024-thread form: no change on C5 / 1 GiB / C2, r4)
    constexpr bool PAIR = BT == 256 && !ZSEG;     // paired launches: the late form (zone_one in 256 threads)
    __shared__ LdsTab<KB_LT> lt;
    __shared__ BodyLds<S, BT, PAIR ? zp_lt<S>() : 1> u;
    // per wave: its sector's new signature bits (the 1024-thread forms: the early,
    // site-heavy merges; the 256-thread late form keeps 4 waves per SIMD without it)
    constexpr bool SIGL = SIG_LDS && BT == 1024;
#ifdef GBPE_NO_SINK
    constexpr bool SINK = false;
#else
    constexpr bool SINK = true;   // body_sector waits for the next sector's prefetch before its stores
#endif
    __shared__ uint32_t s_sig[SIGL ? BT / 64 : 1][SP_SIGW];
    __shared__ uint32_t s_ntok2, s_ntok1, s_n, s_n2, s_any, s_acc, s_rm[BT / 64], s_rm2[BT / 64];
    __shared__ uint32_t s_hit1[PAIR ? SP_CAP / 32 : 1];   // sectors the first merge changed (local index bits)
    __shared__ uint64_t s_mv[BT / 64];
    // the paired form tests a pass's 64 words for each merge (wave 0 the first's
    // rows, wave 1 the second's), into two lists of SP_CAP
    constexpr uint32_t LCAP = (PAIR ? 2u : 1u) * SP_CAP;
    constexpr int QPT = LCAP / BT;   // candidates per thread in the signature test
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (SIGL) s_sig[wid][lane] = 0u;   // (a wave's own words: no barrier needed before its first sector)
#ifdef GBPE_BSPROF
    unsigned long long bsp[6] = {0, 0, 0, 0, 0, 0}, bsp_wall = 0;
#endif
    uint32_t a, b, nw, mc, md;
    Sel2 s2;
    if (t == 0) KT(0);
    const DevState *gs = nullptr, *zs = nullptr;   // this workgroup's snapshots of the states at launch (LDS)
    const Table& xtb = dtb;
    SelShard shx = sh;
    if (!PAIR) shx.k2 = 0u;
    if (!sel_inline<BT, PAIR>(st, zst, part, npart, EXACT, zone1 != 0, tb, log, grpsum, a, b, nw, mc, md, s2, gs, zs, shx)) {
        return;
    }
    if (t == 0) KT(1);
    S* const zcur = (md & 1u) ? zb1 : zb0;   // the zone of merge md
    S* const zoth = (md & 1u) ? zb0 : zb1;
    // the zone workgroup is dispatched first (block 0 when zone1): it is the longest
    // single chain of the merge, and later blocks of a large grid start later
    const uint32_t bid = blockIdx.x - zone1;
    if constexpr (ZSEG) {
        if (blockIdx.x < zone1) {
            zone_seg<S, EXACT, BT, KB_LT, ZPT>(st, zst, *gs, *zs, zcur, zoth, zg, zone1, u.zw.z, lt, dtb, a, b, nw, mc,
                                             wg_bytes + nbody, round);
            if (t == 0) {
                KT(5);
                KTV(6, 2);
            }
            return;
        }
    } else {
        if (zone1 == 1 && blockIdx.x == 0) {
            bool two = false;
            if constexpr (PAIR && !ZP_OFF) {
                if (s2.dbl) {
                    zone_two<S, EXACT, BT, zp_lt<S>(), ZPT>(st, zst, *gs, zs->n, zcur, zoth, zg, u.zw.z, u.zw.wb2,
                                                            u.zw.lt, xtb, a, b, nw, mc, s2, wg_bytes + nbody, round);
                    two = true;
                }
            }
            if (!two)
                zone_one<S, EXACT, BT, KB_LT, ZPT>(st, zst, zs->n, win_src0(*gs, mc), zcur, zoth, u.zw.z, lt, xtb, a, b,
                                                   nw, mc, wg_bytes + nbody, round);
            if (t == 0) {
                KT(5);
                KTV(6, 2);
            }
            return;
        }
    }
    if (bid >= nbody) {
        const uint64_t src0 = win_src0(*gs, mc);
        const uint64_t stride = (uint64_t)(gridDim.x - nbody) * BT;
        for (uint64_t v = (uint64_t)(bid - nbody) * BT + t; v < mc; v += stride) wtmp[v] = zoth[src0 + v];
        if (t == 0) {
            KT(5);
            KTV(6, 3);
        }
        return;
    }
    const bool dbl = PAIR && s2.dbl;   // (block-uniform)
    const uint32_t pid_ab = (a << 16) | b, pid_2 = (s2.a << 16) | s2.b;
    auto& cb = u.c;
    lds_clear(lt);
    if (t == 0) {
        s_any = 0u;
        s_acc = 0u;
    }
    uint32_t removed = 0, removed2 = 0, ncand_all = 0;
    uint64_t moved = 0, rd = 0;   // sector symbols read + rewritten (wave-uniform); extents + signature words read
    // sh.sub > 1: this workgroup takes a 32/sub-sector slice of word bid / sub
    const uint32_t sub = sh.sub, sw = 32u / sub;
    const uint32_t w_beg = sub > 1 ? bid / sub : bid * wpg;
    const uint32_t w_end = sub > 1 ? w_beg + 1 : (w_beg + wpg < W ? w_beg + wpg : W);
    const uint32_t smask = sub > 1 ? ((1u << sw) - 1u) << ((bid % sub) * sw) : 0xFFFFFFFFu;
    // (a paired launch's second merge testing the same 64 words in another wave, not
    // lanes 32-63 of wave 0 over 32 words: C5 1.234 -> 1.146 s, ml1g 0.768 -> 0.750 s —
    // its rows of ~55 words per workgroup took two passes)
    for (uint32_t w0 = w_beg; w0 < w_end; w0 += SP_PW) {
        __syncthreads();   // the previous pass is done with s_ntok* / s_n / the candidate arrays
        if (t == 0) {
            s_ntok2 = 0u;
            s_ntok1 = 0u;
            s_n = 0u;
            s_n2 = 0u;
        }
        if (PAIR && t < (int)(SP_CAP / 32)) s_hit1[t] = 0u;
        __syncthreads();
        // token candidates (a wave per merge: list positions from its scan, no LDS
        // counter): the first merge's rows into [0, SP_CAP), the second's into
        // [SP_CAP, 2 SP_CAP)
        if (t < (int)SP_PW || (dbl && t < 2 * (int)SP_PW)) {
            const bool two = t >= (int)SP_PW;
            const uint32_t w = w0 + (uint32_t)(t & 63);
            const uint32_t ra = two ? s2.a : a, rb = two ? s2.b : b;
            uint32_t c = w < w_end ? bits[(uint64_t)ra * W + w] & bits[(uint64_t)rb * W + w] & smask : 0u;
            const uint32_t pc = (uint32_t)__popc(c), incl = wave_scan_incl_u32(pc);
            uint32_t pos = (two ? SP_CAP : 0u) + incl - pc;
            if ((t & 63) == 63) {
                if (two) s_ntok2 = incl;
                else s_ntok1 = incl;
            }
            while (c) {
                const int bit = __ffs(c) - 1;
                c &= c - 1;
                cb.sec[pos++] = w * 32u + (uint32_t)bit;
            }
        }
        __syncthreads();
        const uint32_t ntok1 = s_ntok1, ntok2 = dbl ? s_ntok2 : 0u, ntok = ntok1 + ntok2;
        if (t == 0) KT(2);
        if (ntok == 0) continue;   // block-uniform
        rd += 16ull * ntok;
        // signature filter: this thread's candidates (their extents load alongside)
        // into registers, then compacted in place (a paired launch: the first merge's
        // from the front, the second's from the back)
        uint32_t cs[QPT];
        uint2 ce[QPT];
        bool ck[QPT];
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            const uint32_t j = (uint32_t)t + (uint32_t)q * BT;
            const bool ok = j < SP_CAP ? j < ntok1 : j - SP_CAP < ntok2;
            cs[q] = ok ? cb.sec[j] : SP_INV;
        }
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            ck[q] = false;
            if (cs[q] != SP_INV) {
                const uint32_t j = (uint32_t)t + (uint32_t)q * BT;
                ce[q] = sec[cs[q]];
                ck[q] = sig_has(sig + (uint64_t)cs[q] * SP_SIGW, j < SP_CAP ? pid_ab : pid_2);
            }
        }
        __syncthreads();   // every candidate is read before the list is rewritten
#pragma unroll
        for (int q = 0; q < QPT; ++q) {   // one LDS counter add per wave, positions from the ballot
            const uint32_t j = (uint32_t)t + (uint32_t)q * BT;
            const bool in2 = PAIR && j >= SP_CAP;
            const unsigned long long m = __ballot(ck[q] && !in2);
            uint32_t base = 0;
            if (lane == 0 && m) base = atomicAdd(&s_n, (uint32_t)__popcll(m));
            base = __builtin_amdgcn_readlane(base, 0);
            if (ck[q] && !in2) {
                const uint32_t qq = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                cb.sec[qq] = cs[q];
                cb.ext[qq] = ce[q];
            }
            if (PAIR) {
                const unsigned long long m2 = __ballot(ck[q] && in2);
                uint32_t base2 = 0;
                if (lane == 0 && m2) base2 = atomicAdd(&s_n2, (uint32_t)__popcll(m2));
                base2 = __builtin_amdgcn_readlane(base2, 0);
                if (ck[q] && in2) {
                    const uint32_t qq = LCAP - 1u - base2 -
                                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m2, 0u));
                    cb.sec[qq] = cs[q];
                    cb.ext[qq] = ce[q];
                }
            }
        }
        __syncthreads();
        const uint32_t n1 = s_n, n2 = PAIR ? s_n2 : 0u;
        if (t == 0) KT(3);
        if (n1 + n2 == 0) continue;   // block-uniform
        ncand_all += n1 + n2;
        if (t == 0) s_any = 1u;
#pragma unroll 1
        for (int ph = 0; ph < (PAIR ? 2 : 1); ++ph) {   // the first merge's sectors, then the second's
            const uint32_t ncand = ph ? n2 : n1;
            if (ph) {
                if (t == 0) KT(10);
                if (ncand == 0) break;   // block-uniform
                // the first merge's sector stores land before the second reads them back; in
                // ref mode the zone workgroup's verdict first (it never waits on a body workgroup)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (t == 0) {
                    uint32_t v = 3u;
                    if (!EXACT) {
                        const uint32_t tag = gs->epoch << 2;
                        for (uint32_t it = 0;; ++it) {
                            v = __hip_atomic_load(pair_word(zg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if ((v & ~3u) == tag && (v & 2u)) break;
                            if (it > ZSEG_SPIN) {
                                atomicOr(&st->err, ERR_SPIN);
                                v = 2u;
                                break;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                    s_acc = v & 1u;
                }
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (t == 0) KT(11);
                if (!s_acc) break;   // block-uniform
            }
            const uint32_t base = ph ? LCAP - ncand : 0u;   // (the second list is stored backwards: any order)
            const uint32_t ca = ph ? s2.a : a, cbb = ph ? s2.b : b, cn = ph ? nw + 1u : nw;
            // a sector the first merge changed in this workgroup: its extent is re-read
            auto ext_of = [&](uint32_t j) -> uint2 {
                const uint32_t sct = cb.sec[base + j];
                if (PAIR && ph && ((s_hit1[(sct - w0 * 32u) >> 5] >> (sct & 31u)) & 1u)) {
                    const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&sec[sct]), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
                }
                return cb.ext[base + j];
            };
            // software-pipelined: a wave's next sector loads while it merges this one
            uint32_t nf[5], nfm[4];
#ifdef GBPE_BSPROF
            const unsigned long long sp0 = clock64();
#endif
            uint2 en = make_uint2(0u, 0u);
            if ((uint32_t)wid < ncand) {
                en = ext_of((uint32_t)wid);
                sector_first<S>(body + en.x, lmul ? lmul + en.x : nullptr, en.y, nf, nfm);
            }
            for (uint32_t j = wid; j < ncand; j += BT / 64) {
                const uint32_t sct = cb.sec[base + j];
                const uint2 e = en;
                uint32_t cf[5], cfm[4];
#pragma unroll
                for (int k = 0; k < 5; ++k) cf[k] = nf[k];
#pragma unroll
                for (int k = 0; k < 4; ++k) cfm[k] = nfm[k];
                if (j + BT / 64 < ncand) {
                    en = ext_of(j + BT / 64);
                    sector_first<S>(body + en.x, lmul ? lmul + en.x : nullptr, en.y, nf, nfm);
                }
                uint32_t out = 0;
                const uint32_t r = body_sector<S, KB_LT, Table, LdsTab<KB_LT>, SIGL>(
                    body + e.x, lmul ? lmul + e.x : nullptr, e.y, ca, cbb, cn, lt, xtb, st, sig + (uint64_t)sct * SP_SIGW,
                    out, cf, cfm, s_sig[SIGL ? wid : 0], SINK ? nf : nullptr, SINK ? nfm : nullptr BSP_PASS);
                moved += (uint64_t)(sizeof(S) + (lmul ? 4u : 0u)) * (e.y + (r ? out : 0u));
                if (r) {
                    if (ph) removed2 += r;
                    else removed += r;
                    if (lane == 0) {
                        if (clog) atomicAdd(&st->hitsec, 1u);
                        sec[sct].y = out;
                        atomicOr(&bits[(uint64_t)cn * W + (sct >> 5)], 1u << (sct & 31u));
                        if (PAIR && dbl && !ph) atomicOr(&s_hit1[(sct - w0 * 32u) >> 5], 1u << (sct & 31u));
                    }
                }
            }
#ifdef GBPE_BSPROF
            bsp_wall += clock64() - sp0;
#endif
            if (PAIR && dbl && !ph) __syncthreads();   // s_hit1 complete before the second merge's extents
        }
    }
#ifdef GBPE_BSPROF
    if (lane == 0) {
        for (int k = 0; k < 6; ++k) atomicAdd(&g_bsprof[k], bsp[k]);
        atomicAdd(&g_bsprof[6], bsp_wall);
        atomicAdd(&g_bsprof[7], 1ull);
    }
#endif
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
    lds_flush(lt, xtb, st);
    if (lane == 0) {
        s_rm[wid] = removed;
        s_rm2[wid] = removed2;
        s_mv[wid] = moved;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t r = 0, r2 = 0;
        uint64_t mv = rd;
        for (int w2 = 0; w2 < BT / 64; ++w2) {
            r += s_rm[w2];
            r2 += s_rm2[w2];
            mv += s_mv[w2];
        }
        if (r) atomicAdd(&st->body_rm, r);
        if (r2) atomicAdd(&st->body_rm2, r2);
        atomicAdd(&wg_bytes[bid], mv);   // this workgroup's own counter
        KT(5);
        KTV(6, 1 | (ncand_all << 8));
    }
}

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
