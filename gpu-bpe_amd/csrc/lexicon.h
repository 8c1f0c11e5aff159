// Word-lexicon body of the sector-sparse loop.  Included by
// train.hip inside its anonymous namespace (uses Sym, TILE, TPB, EPT, SP_INV).
//
// No counted pair ever spans a word start (train.wgsl:395, 483, 493) or holds
// token 0, and 0 tokens never merge, so the body is a multiset of WORDS: two
// occurrences with the same symbols merge identically at every merge.  The
// body is therefore kept as one copy of every distinct word (the "store"),
// each followed by a 0 separator (which, like a word start, blocks every
// pair), with a per-symbol multiplicity array.  A merge then touches each
// distinct word once and weights its count deltas by the word's multiplicity:
// the pair counts stay exactly the stream's (1 GiB English: ~3*10^8 words,
// ~2*10^5 distinct).  The stream order lives in an occurrence list (one uid or
// literal per body word), expanded back to the dense stream on exit/export.
// The reference compaction quirk only ever acts on the stream's tail, which
// stays in the dense zone.

constexpr uint32_t LX_LIT = 0x80000000u;   // occurrence of a token-0 symbol: the symbol itself (low bits)
constexpr uint32_t LX_LONG = 0x40000000u;  // build only: a word longer than LX_LMAX (index into the long list)
constexpr uint32_t LX_LMAX = 64;           // words up to this many symbols are deduplicated
constexpr int LX_WPT = 16;                 // words per thread in k_lx_hash (at least; trainer lx_wg)
constexpr int LX_LT = 2048;                // LDS word-table slots per workgroup (a multiple of TPB)
constexpr uint32_t LX_PROBES = 4096;       // global word-table probes before the build gives up

// a body word starts at i iff no counted pair can ever span (i-1, i)
template <typename S>
__device__ __forceinline__ bool lx_is_start(uint32_t prev, uint32_t cur, bool first) {
    return first || (cur & Sym<S>::WS) || !(cur & Sym<S>::TM) || !(prev & Sym<S>::TM);
}

// per 8192-symbol tile: number of word starts
template <typename S>
__global__ __launch_bounds__(TPB) void k_lx_count(const S* __restrict__ x, uint32_t len, uint32_t* __restrict__ tilecnt) {
    __shared__ uint32_t s[TPB / 64];
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    uint32_t c = 0;
#pragma unroll 4
    for (int k = 0; k < EPT; ++k) {
        const uint64_t i = base + (uint64_t)k * TPB + threadIdx.x;
        if (i < len) c += lx_is_start<S>(i ? (uint32_t)x[i - 1] : 0u, (uint32_t)x[i], i == 0) ? 1u : 0u;
    }
    c = wave_sum_u32(c);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < TPB / 64; ++w) t += s[w];
        tilecnt[blockIdx.x] = t;
    }
}

// word start positions in stream order (tile prefix from k_chunk_scan1/2)
template <typename S>
__global__ __launch_bounds__(TPB) void k_lx_wpos(const S* __restrict__ x, uint32_t len, const uint32_t* __restrict__ tpre,
                                                 const uint64_t* __restrict__ tblk, uint32_t* __restrict__ wpos) {
    __shared__ uint32_t pre[EPT * (TPB / 64)];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    uint32_t f = 0;   // bit k: position base + k*TPB + threadIdx.x starts a word
#pragma unroll 4
    for (int k = 0; k < EPT; ++k) {
        const uint64_t i = base + (uint64_t)k * TPB + threadIdx.x;
        const bool st = i < len && lx_is_start<S>(i ? (uint32_t)x[i - 1] : 0u, (uint32_t)x[i], i == 0);
        f |= (st ? 1u : 0u) << k;
        const unsigned long long m = __ballot(st);
        if (lane == 0) pre[k * (TPB / 64) + wid] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = tpre[blockIdx.x] + (uint32_t)tblk[blockIdx.x / SCAN_BLK];
        for (int q = 0; q < EPT * (TPB / 64); ++q) {
            const uint32_t v = pre[q];
            pre[q] = run;
            run += v;
        }
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int k = 0; k < EPT; ++k) {
        const bool st = (f >> k) & 1u;
        const unsigned long long m = __ballot(st);
        if (st) wpos[pre[k * (TPB / 64) + wid] + (uint32_t)__popcll(m & lt)] = (uint32_t)(base + (uint64_t)k * TPB + threadIdx.x);
    }
}

// 64-bit content hash of a word (its symbols with their word-start bits, and its length)
// (8 symbols' loads issued together: one round trip per 8 symbols, not per symbol)
template <typename S>
__device__ __forceinline__ unsigned long long lx_hash(const S* __restrict__ x, uint32_t s, uint32_t L) {
    unsigned long long h = 0x9E3779B97F4A7C15ull ^ (unsigned long long)L;
    for (uint32_t i0 = 0; i0 < L; i0 += 8) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i0 + k < L ? (uint32_t)x[s + i0 + k] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (i0 + k >= L) break;
            h ^= (unsigned long long)v[k];
            h *= 0x100000001B3ull;
            h ^= h >> 29;
        }
    }
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h ? h : 1ull;
}

__device__ __forceinline__ uint32_t lx_home(unsigned long long h, uint32_t mask) { return (uint32_t)(h ^ (h >> 32)) & mask; }

// Word-table slot: the 64-bit key with its value in the same 16 bytes, so a
// probe's one line fetch brings both (the table is far larger than the caches
// at 1 GiB, and separate key / value arrays cost two random lines per word).
struct alignas(16) LxSlot {
    unsigned long long key;   // 0 = empty
    uint32_t rep;             // a representative occurrence (word index)
    uint32_t cnt;             // occurrences; the uid once k_lx_tabuid ran
};

// The word table is cut into slices (at most 256, of >= 4096 slots unless the table is
// smaller) and a probe sequence wraps inside its home slot's slice: the two-stage
// build (k_lx_hash's bucketed flush + k_lx_fold) gives every slice one workgroup.
__device__ __forceinline__ uint32_t lx_slice(uint32_t P) { return P >= (1u << 20) ? P >> 8 : (P < 4096u ? P : 4096u); }
__device__ __forceinline__ uint32_t lx_next(uint32_t slot, uint32_t sm) { return (slot & ~sm) | ((slot + 1u) & sm); }
__device__ __forceinline__ uint32_t lx_bucket(unsigned long long h, uint32_t P) {
    return lx_home(h, P - 1) / lx_slice(P);
}

// global word table (linear probing on 64-bit keys, inside the home slice): insert-or-add
// `c` occurrences.  A key never changes once set (0 -> h), so the probes are plain loads
// that may hit a stale copy in this XCD's L2: a stale 0 only sends the probe to the CAS,
// which returns the key actually there (agent-scope probe loads go to memory).
__device__ bool lx_insert(LxSlot* __restrict__ wt, uint32_t P, unsigned long long h, uint32_t rep, uint32_t c,
                          uint32_t maxp = LX_PROBES) {
    const uint32_t sm = lx_slice(P) - 1u;
    uint32_t slot = lx_home(h, P - 1);
    if (maxp > sm + 1u) maxp = sm + 1u;
    for (uint32_t p = 0; p < maxp; ++p, slot = lx_next(slot, sm)) {
        unsigned long long k = wt[slot].key;
        if (k == 0ull) {
            k = atomicCAS(&wt[slot].key, 0ull, h);
            if (k == 0ull) {
                wt[slot].rep = rep;   // any occurrence represents the word
                atomicAdd(&wt[slot].cnt, c);
                return true;
            }
        }
        if (k == h) {
            atomicAdd(&wt[slot].cnt, c);
            return true;
        }
    }
    return false;
}

// the slot of key h (its whole 16 bytes in one load), or SP_INV in .z
__device__ uint4 lx_find(const LxSlot* __restrict__ wt, uint32_t P, unsigned long long h) {
    const uint32_t sm = lx_slice(P) - 1u;
    uint32_t slot = lx_home(h, P - 1);
    for (uint32_t p = 0; p <= sm && p < LX_PROBES; ++p, slot = lx_next(slot, sm)) {
        const uint4 v = *reinterpret_cast<const uint4*>(&wt[slot]);
        const unsigned long long k = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
        if (k == h) return v;
        if (k == 0ull) break;
    }
    return make_uint4(0u, 0u, SP_INV, SP_INV);
}

// Word multiplicities: every workgroup aggregates TPB x wpt words in an LDS table
// (hot words cost one global add per workgroup, not one per occurrence), then
// adds them into the global table (the host sizes wpt for ~lx_wg workgroups).
// Those global adds are most of the kernel (1 GiB: 9.3 ms, 3.2 without them), and
// their number barely moves with the workgroup size: 62K workgroups of 4096
// words or 1024 of 247K words (whose LDS tables overflow into direct inserts)
// measured 9.4 vs 10.1 ms (profiles/r5/s9).  Token-0 words become literals, long words
// entries of their own.  ctr[0] = long words, ctr[1] = failure flag.
// wmul (weighted analysis, the lexicon hand-over of DESIGN §5): a word counts
// wmul[its first position] occurrences instead of one — the segment is then a
// concatenation of word stores, each word carrying its multiplicity.
// rec (the two-stage build of a large segment; launched as 1,024-thread
// workgroups with an 8,192-slot LDS table, so a workgroup's distinct words fit it and
// do not overflow into global inserts): instead of adding its entries to the global
// table, the workgroup writes them as LxSlot records to its own region
// rec[blockIdx.x * LT ...], grouped by word-table slice (bucket), with the groups'
// offsets and sizes in bmeta[0 / 1][blockIdx.x * nbk + bucket]; k_lx_fold then folds
// every bucket in one workgroup's LDS and inserts each distinct word once.
template <typename S, int BT = TPB, int LT = LX_LT>
__global__ __launch_bounds__(BT) void k_lx_hash(const S* __restrict__ x, uint32_t len, const uint32_t* __restrict__ wpos,
                                                 uint32_t nw, LxSlot* __restrict__ wtab,
                                                 uint32_t P, uint32_t* __restrict__ otmp, uint32_t* __restrict__ longs,
                                                 uint32_t* __restrict__ ctr, const uint32_t* __restrict__ wmul,
                                                 uint32_t maxp, uint32_t wpt, LxSlot* __restrict__ rec = nullptr,
                                                 uint32_t* __restrict__ bmeta = nullptr, uint32_t nbk = 0,
                                                 uint32_t nwg = 0) {
    __shared__ unsigned long long lk[LT];
    __shared__ uint32_t lc[LT], lr[LT];
    for (int i = threadIdx.x; i < LT; i += BT) {
        lk[i] = 0ull;
        lc[i] = 0u;
    }
    __syncthreads();
    const uint64_t j0 = (uint64_t)blockIdx.x * BT * wpt;
    for (uint32_t q = 0; q < wpt; ++q) {
        const uint64_t j = j0 + (uint64_t)q * BT + threadIdx.x;
        if (j >= nw) break;
        const uint32_t s = wpos[j], e = j + 1 < nw ? wpos[j + 1] : len, L = e - s;
        const uint32_t v0 = x[s];
        if (!(v0 & Sym<S>::TM)) {
            otmp[j] = LX_LIT | v0;
            continue;
        }
        if (L > LX_LMAX) {
            const uint32_t li = atomicAdd(&ctr[0], 1u);
            longs[li] = (uint32_t)j;
            otmp[j] = LX_LONG | li;
            continue;
        }
        otmp[j] = 0u;
        const uint32_t wt = wmul ? wmul[s] : 1u;
        const unsigned long long h = lx_hash<S>(x, s, L);
        uint32_t slot = lx_home(h, LT - 1);
        bool done = false;
        for (int p = 0; p < 32 && !done; ++p, slot = (slot + 1) & (LT - 1)) {
            const unsigned long long o = atomicCAS(&lk[slot], 0ull, h);
            if (o == 0ull) {
                lr[slot] = (uint32_t)j;
                atomicAdd(&lc[slot], wt);
                done = true;
            } else if (o == h) {
                atomicAdd(&lc[slot], wt);
                done = true;
            }
        }
        if (!done && !lx_insert(wtab, P, h, (uint32_t)j, wt, maxp)) ctr[1] = 1u;
    }
    __syncthreads();
    constexpr int FL = LT / BT;
    if (rec) {   // two-stage: the entries as records, grouped by bucket (k_lx_fold adds them)
        __shared__ uint32_t s_bc[256], s_bo[256], s_ws[BT / 64];
        for (uint32_t i = threadIdx.x; i < 256; i += BT) s_bc[i] = 0u;
        __syncthreads();
        unsigned long long fk[FL];
        uint32_t bk[FL], rk[FL];
#pragma unroll
        for (int q = 0; q < FL; ++q) {
            fk[q] = lk[threadIdx.x + q * BT];
            bk[q] = fk[q] ? lx_bucket(fk[q], P) : 0u;
            rk[q] = fk[q] ? atomicAdd(&s_bc[bk[q]], 1u) : 0u;
        }
        __syncthreads();
        {   // exclusive scan of the bucket sizes (nbk <= 256 = BT: one per thread)
            const uint32_t v = threadIdx.x < nbk ? s_bc[threadIdx.x] : 0u;
            const uint32_t incl = wave_scan_incl_u32(v);
            if ((threadIdx.x & 63) == 63) s_ws[threadIdx.x >> 6] = incl;
            __syncthreads();
            uint32_t pre = incl - v;
            for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += s_ws[w];
            if (threadIdx.x < nbk) {
                s_bo[threadIdx.x] = pre;
                bmeta[(uint64_t)blockIdx.x * nbk + threadIdx.x] = pre;
                bmeta[(uint64_t)nwg * nbk + (uint64_t)blockIdx.x * nbk + threadIdx.x] = v;
            }
        }
        __syncthreads();
        LxSlot* r = rec + (uint64_t)blockIdx.x * LT;
#pragma unroll
        for (int q = 0; q < FL; ++q) {
            if (!fk[q]) continue;
            const int i = threadIdx.x + q * BT;
            *reinterpret_cast<uint4*>(&r[s_bo[bk[q]] + rk[q]]) =
                make_uint4((uint32_t)fk[q], (uint32_t)(fk[q] >> 32), lr[i], lc[i]);
        }
        return;
    }
    // a table already known to be too small (the build is redone or abandoned): no probing
    if (__hip_atomic_load(&ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    // the thread's LT / BT entries: every home-slot probe issued together, the
    // adds of the words found there last (no later load waits behind them)
    unsigned long long fk[FL], hk[FL];
    uint32_t fs[FL];
#pragma unroll
    for (int q = 0; q < FL; ++q) {
        fk[q] = lk[threadIdx.x + q * BT];
        fs[q] = lx_home(fk[q], P - 1);
        hk[q] = fk[q] ? wtab[fs[q]].key : 0ull;
    }
    bool home[FL];
#pragma unroll
    for (int q = 0; q < FL; ++q) {
        const int i = threadIdx.x + q * BT;
        home[q] = fk[q] && hk[q] == fk[q];
        if (fk[q] && !home[q] && !lx_insert(wtab, P, fk[q], lr[i], lc[i], maxp)) ctr[1] = 1u;
    }
#pragma unroll
    for (int q = 0; q < FL; ++q)
        if (home[q]) atomicAdd(&wtab[fs[q]].cnt, lc[threadIdx.x + q * BT]);
}

// Second stage of the two-stage build: bucket blockIdx.x's records of every
// k_lx_hash workgroup, folded in LDS (a word repeated across workgroups becomes one
// entry), then inserted into the bucket's own slice of the word table — no other
// workgroup touches it, so the inserts do not contend.  A full LDS table sends the
// record straight to the global table.  Each thread takes whole workgroup groups,
// their sizes loaded FOLD_B at a time and their records FOLD_R at a time.
constexpr int FOLD_T = 1024, FOLD_LT = 8192, FOLD_B = 8, FOLD_R = 8;
__global__ __launch_bounds__(FOLD_T) void k_lx_fold(const LxSlot* __restrict__ rec, const uint32_t* __restrict__ bmeta,
                                                    uint32_t nwg, uint32_t nbk, LxSlot* __restrict__ wtab, uint32_t P,
                                                    uint32_t* __restrict__ ctr, uint32_t maxp, uint32_t rstride) {
    __shared__ unsigned long long fk[FOLD_LT];
    __shared__ uint32_t fc[FOLD_LT], fr[FOLD_LT];
    if (__hip_atomic_load(&ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;   // (stage 1 gave up)
    for (int i = threadIdx.x; i < FOLD_LT; i += FOLD_T) {
        fk[i] = 0ull;
        fc[i] = 0u;
    }
    __syncthreads();
    const uint32_t b = blockIdx.x;
    bool fail = false;
    for (uint32_t w0 = threadIdx.x; w0 < nwg; w0 += FOLD_T * FOLD_B) {
        uint32_t st[FOLD_B], n[FOLD_B];
#pragma unroll
        for (int k = 0; k < FOLD_B; ++k) {
            const uint32_t w = w0 + (uint32_t)k * FOLD_T;
            st[k] = w < nwg ? bmeta[(uint64_t)w * nbk + b] : 0u;
            n[k] = w < nwg ? bmeta[(uint64_t)nwg * nbk + (uint64_t)w * nbk + b] : 0u;
        }
#pragma unroll 1
        for (int k = 0; k < FOLD_B; ++k) {
            const uint4* r = reinterpret_cast<const uint4*>(rec + (uint64_t)(w0 + (uint32_t)k * FOLD_T) * rstride + st[k]);
            for (uint32_t i0 = 0; i0 < n[k]; i0 += FOLD_R) {
                uint4 v[FOLD_R];
#pragma unroll
                for (int q = 0; q < FOLD_R; ++q) v[q] = i0 + q < n[k] ? r[i0 + q] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (int q = 0; q < FOLD_R; ++q) {
                    const unsigned long long h = (unsigned long long)v[q].x | ((unsigned long long)v[q].y << 32);
                    if (!h) continue;
                    uint32_t slot = lx_home(h, FOLD_LT - 1);
                    bool done = false;
                    for (int p = 0; p < 64 && !done; ++p, slot = (slot + 1) & (FOLD_LT - 1)) {
                        const unsigned long long o = atomicCAS(&fk[slot], 0ull, h);
                        if (o == 0ull) fr[slot] = v[q].z;
                        if (o == 0ull || o == h) {
                            atomicAdd(&fc[slot], v[q].w);
                            done = true;
                        }
                    }
                    if (!done && !lx_insert(wtab, P, h, v[q].z, v[q].w, maxp)) fail = true;
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < FOLD_LT; i += FOLD_T)
        if (fk[i] && !lx_insert(wtab, P, fk[i], fr[i], fc[i], maxp)) fail = true;
    if (fail) ctr[1] = 1u;
}

constexpr uint32_t LX_TB = TPB * 16;   // word-table slots per uid-assignment block

// slot k of thread t in block b: b * LX_TB + k * TPB + t (lane-contiguous, so every
// load instruction of a wave reads 1 KB in one piece)
__device__ __forceinline__ uint64_t lx_tslot(uint32_t k) { return (uint64_t)blockIdx.x * LX_TB + (uint64_t)k * TPB + threadIdx.x; }

__global__ __launch_bounds__(TPB) void k_lx_tabcount(const LxSlot* __restrict__ wt, uint32_t P, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t s[TPB / 64];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = lx_tslot(k);
        c += (i < P && wt[i].key) ? 1u : 0u;
    }
    c = wave_sum_u32(c);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < TPB / 64; ++w) t += s[w];
        cnt[blockIdx.x] = t;
    }
}

// word length of word j of the segment
__device__ __forceinline__ uint32_t lx_wlen(const uint32_t* __restrict__ wpos, uint32_t nw, uint32_t len, uint32_t j) {
    return (j + 1 < nw ? wpos[j + 1] : len) - wpos[j];
}

// uids by block, then thread, then the thread's slots (lx_tslot): usz = length + 1
// (its separator), umul = occurrences, urep = a representative's position; the
// slot's count becomes the uid
__global__ __launch_bounds__(TPB) void k_lx_tabuid(LxSlot* __restrict__ wt, uint32_t P, const uint32_t* __restrict__ bpre,
                                                   const uint64_t* __restrict__ bblk, const uint32_t* __restrict__ wpos,
                                                   uint32_t nw, uint32_t len, uint32_t* __restrict__ usz,
                                                   uint32_t* __restrict__ umul, uint32_t* __restrict__ urep) {
    __shared__ uint32_t s[TPB / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t occ = 0;
    uint2 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = lx_tslot(k);
        const uint4 e = i < P ? *reinterpret_cast<const uint4*>(&wt[i]) : make_uint4(0u, 0u, 0u, 0u);
        v[k] = make_uint2(e.z, e.w);
        occ |= ((e.x | e.y) ? 1u : 0u) << k;
    }
    const uint32_t c = (uint32_t)__popc(occ);
    const uint32_t incl = wave_scan_incl_u32(c);
    if (lane == 63) s[wid] = incl;
    __syncthreads();
    uint32_t u = bpre[blockIdx.x] + (uint32_t)bblk[blockIdx.x / SCAN_BLK] + incl - c;
    for (int w = 0; w < wid; ++w) u += s[w];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (!((occ >> k) & 1u)) continue;
        usz[u] = lx_wlen(wpos, nw, len, v[k].x) + 1u;
        umul[u] = v[k].y;
        urep[u] = wpos[v[k].x];
        wt[lx_tslot(k)].cnt = u;
        ++u;
    }
}

// long words: an entry each (uids after the deduplicated ones)
__global__ void k_lx_longs(const uint32_t* __restrict__ longs, const uint32_t* __restrict__ ctr, uint32_t nshort,
                           const uint32_t* __restrict__ wpos, uint32_t nw, uint32_t len, uint32_t* __restrict__ usz,
                           uint32_t* __restrict__ umul, uint32_t* __restrict__ urep,
                           const uint32_t* __restrict__ wmul = nullptr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ctr[0]) return;
    const uint32_t j = longs[i];
    usz[nshort + i] = lx_wlen(wpos, nw, len, j) + 1u;
    umul[nshort + i] = wmul ? wmul[wpos[j]] : 1u;
    urep[nshort + i] = wpos[j];
}

// store layout: word u at off(u) (scanned sizes), its separator after it; the
// multiplicity of every symbol (0 for separators; mul null: symbols only)
template <typename S>
__global__ void k_lx_fill(const S* __restrict__ x, const uint32_t* __restrict__ urep, const uint32_t* __restrict__ usz,
                          const uint32_t* __restrict__ umul, const uint32_t* __restrict__ upre,
                          const uint64_t* __restrict__ ublk, uint32_t nu, S* __restrict__ store, uint32_t* __restrict__ mul) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nu) return;
    const uint32_t off = upre[u] + (uint32_t)ublk[u / SCAN_BLK], L = usz[u] - 1u, r = urep[u], m = umul[u];
    for (uint32_t i = 0; i < L; ++i) {
        store[off + i] = x[r + i];
        if (mul) mul[off + i] = m;
    }
    store[off + L] = (S)0;
    if (mul) mul[off + L] = 0u;
}

// sector windows over the new store region [sbase, sbase + T): window k's
// sector starts at its first word (starts[] preset to SP_INV); w0 = its first uid
__global__ void k_lx_secstart(const uint32_t* __restrict__ upre, const uint64_t* __restrict__ ublk, uint32_t nu,
                              uint32_t SEC, uint32_t sbase, uint32_t uid_base, uint32_t* __restrict__ starts,
                              uint32_t* __restrict__ w0) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nu) return;
    const uint32_t o = upre[u] + (uint32_t)ublk[u / SCAN_BLK], k = o / SEC;
    const bool first = u == 0 || (upre[u - 1] + (uint32_t)ublk[(u - 1) / SCAN_BLK]) / SEC != k;
    if (first) {
        starts[k] = sbase + o;
        w0[k] = uid_base + u;
    }
}

// occurrence list of the segment's words (stream order): the uid of each word,
// after checking its symbols against the representative's (a hash collision
// fails the build instead of merging two different words)
// The symbols are checked against the entries' compact copy (rstore, laid out as
// the store: entry u at upre[u] + ublk[u / SCAN_BLK]), which stays in the caches;
// a representative's occurrence in the segment is a random HBM line per word
// (3.7 of the 1 GiB build's 7.7 ms).
template <typename S>
__global__ void k_lx_occ(const S* __restrict__ x, const uint32_t* __restrict__ wpos, uint32_t nw, uint32_t len,
                         const uint32_t* __restrict__ otmp, const LxSlot* __restrict__ wt,
                         uint32_t P, const S* __restrict__ rstore, const uint32_t* __restrict__ upre,
                         const uint64_t* __restrict__ ublk,
                         const uint32_t* __restrict__ usz, uint32_t nshort, uint32_t uid_base, uint32_t* __restrict__ occ,
                         uint32_t* __restrict__ ctr) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nw) return;
    const uint32_t o = otmp[j];
    if (o & LX_LIT) {
        occ[j] = o;
        return;
    }
    if (o & LX_LONG) {
        occ[j] = uid_base + nshort + (o & ~LX_LONG);
        return;
    }
    const uint32_t s = wpos[j], L = lx_wlen(wpos, nw, len, (uint32_t)j);
    const uint4 e = lx_find(wt, P, lx_hash<S>(x, s, L));
    bool ok = (e.x | e.y) != 0u;
    uint32_t u = 0;
    if (ok) {
        u = e.w;
        ok = usz[u] == L + 1u;
        const S* r = rstore + upre[u] + ublk[u / SCAN_BLK];
        for (uint32_t i0 = 0; ok && i0 < L; i0 += 8) {
            uint32_t va[8], vb[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                va[k] = i0 + k < L ? (uint32_t)r[i0 + k] : 0u;
                vb[k] = i0 + k < L ? (uint32_t)x[s + i0 + k] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) ok = ok && va[k] == vb[k];
        }
    }
    if (!ok) ctr[1] = 1u;
    occ[j] = uid_base + u;
}

// ── store → stream (sparse exit, symbol export) ──

// current offset and length of every word, from the separators (one wave per sector)
template <typename S>
__global__ __launch_bounds__(TPB) void k_lx_wordpos(const S* __restrict__ store, const uint2* __restrict__ sec,
                                                    uint32_t nsec, const uint32_t* __restrict__ w0,
                                                    uint32_t* __restrict__ coff, uint32_t* __restrict__ clen) {
    const uint32_t k = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nsec) return;
    const uint2 e = sec[k];
    if (!e.y) return;
    uint32_t uid = w0[k], cs = e.x;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t c0 = 0; c0 < e.y; c0 += 64) {
        const uint32_t i = e.x + c0 + (uint32_t)lane;
        const bool sep = c0 + (uint32_t)lane < e.y && store[i] == (S)0;
        const unsigned long long m = __ballot(sep);
        if (sep) {
            const unsigned long long below = m & lt;
            const uint32_t st0 = below ? e.x + c0 + (uint32_t)(63 - __clzll((long long)below)) + 1u : cs;
            const uint32_t u = uid + (uint32_t)__popcll(below);
            coff[u] = st0;
            clen[u] = i - st0;
        }
        uid += (uint32_t)__popcll(m);
        if (m) cs = e.x + c0 + (uint32_t)(63 - __clzll((long long)m)) + 1u;
    }
}

// bad (optional): set when an occurrence names no entry (o >= nu); it then counts 0 symbols
__global__ void k_lx_olen(const uint32_t* __restrict__ occ, uint64_t nocc, const uint32_t* __restrict__ clen,
                          uint32_t* __restrict__ olen, uint32_t nu = 0xFFFFFFFFu, uint32_t* __restrict__ bad = nullptr) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nocc) return;
    const uint32_t o = occ[j];
    if (!(o & LX_LIT) && o >= nu) {
        if (bad) *bad = 1u;
        olen[j] = 0u;
        return;
    }
    olen[j] = (o & LX_LIT) ? 1u : clen[o];
}

template <typename S>
__global__ void k_lx_expand(const uint32_t* __restrict__ occ, uint64_t nocc, const uint32_t* __restrict__ coff,
                            const uint32_t* __restrict__ clen, const S* __restrict__ store,
                            const uint32_t* __restrict__ opre, const uint64_t* __restrict__ oblk, S* __restrict__ dst,
                            uint32_t nu) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nocc) return;
    const uint64_t off = (uint64_t)opre[j] + oblk[j / SCAN_BLK];
    const uint32_t o = occ[j];
    if (o & LX_LIT) {
        dst[off] = (S)(o & ((Sym<S>::WS << 1) - 1u));
        return;
    }
    if (o >= nu) return;   // (k_lx_olen reported it; the host stops before this kernel)
    const uint32_t c = coff[o], L = clen[o];
    for (uint32_t i = 0; i < L; ++i) dst[off + i] = store[c + i];
}
