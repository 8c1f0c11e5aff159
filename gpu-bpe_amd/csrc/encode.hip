// Chunked greedy longest-match trie encode on MI355X (gfx950).
//
// Replaces tokenize.wgsl (trie_tokenizer_chunked :88-175, trie_prefix_sum
// :199-208, trie_tokenizer_compact :225-243) and the TrieTokenizer host
// pass (tokenizer.js:213-335).
//
// Layout: the reference walks a BFS trie of {firstChild, numChildren,
// tokenId} nodes with a binary search over sorted edges per byte
// (tokenize.wgsl:69-86: up to 8 dependent loads per byte).  On upload we
// recompile the same trie into a double-array table: state t's record is
// {check = parent state, base, tokenId}, and the child of state s on byte c
// is t = base(s) + c iff record[t].check == s — one 16-byte L2-resident load
// per byte consumed.  The 256 root transitions (and their depth-1 records)
// live in LDS, as in the reference's root LUT + depth-1 cache
// (tokenize.wgsl:51-63, 93-119).  Transitions are identical to the
// reference trie's, so token ids are bit-identical.

#include "common.h"
#include "scan.h"

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

namespace {

constexpr int WALK_TPB = 256;
constexpr uint64_t kEncSlice = 128ull << 20;   // gbpe_encode's pipeline slice (host buffers)
constexpr uint32_t INV = 0xFFFFFFFFu;

template <typename T>
__global__ __launch_bounds__(WALK_TPB) void k_trie_walk(const uint8_t* __restrict__ in, uint64_t n, uint32_t cs,
                                                        const uint4* __restrict__ rec, uint32_t nrec,
                                                        const uint4* __restrict__ root, T* __restrict__ scratch,
                                                        uint32_t* __restrict__ counts, uint64_t nchunks) {
    __shared__ uint4 lut[256];   // byte -> {state, base, tokenId, present}
    lut[threadIdx.x] = root[threadIdx.x];
    __syncthreads();
    const uint64_t chunk = (uint64_t)blockIdx.x * WALK_TPB + threadIdx.x;
    if (chunk >= nchunks) return;
    const uint64_t c0 = chunk * cs;
    const uint64_t ce = min(c0 + cs, n);
    T* out = scratch + c0;
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
    uint64_t widx = ~0ull;
    uint32_t word = 0;
    auto byte_at = [&](uint64_t p) -> uint32_t {
        const uint64_t wi = p >> 2;
        if (wi != widx) {
            word = in32[wi];
            widx = wi;
        }
        return (word >> ((p & 3u) * 8u)) & 0xFFu;
    };
    uint32_t cnt = 0;
    uint64_t pos = c0;
    while (pos < ce) {
        const uint32_t c = byte_at(pos);
        const uint4 e = lut[c];
        uint32_t lmt = INV;
        uint64_t lmp = pos;
        if (e.w) {
            uint32_t s = e.x, base = e.y;
            if (e.z != INV) {
                lmt = e.z;
                lmp = pos + 1;
            }
            uint64_t wp = pos + 1;
            while (wp < ce) {
                const uint32_t t = base + byte_at(wp);
                if (t >= nrec) break;
                const uint4 r = rec[t];
                if (r.x != s) break;
                s = t;
                base = r.y;
                ++wp;
                if (r.z != INV) {
                    lmt = r.z;
                    lmp = wp;
                }
            }
        }
        if (lmt != INV) {
            out[cnt++] = (T)lmt;
            pos = lmp;
        } else {   // no token starts here: emit the raw byte value (tokenize.wgsl:169-171)
            out[cnt++] = (T)c;
            ++pos;
        }
    }
    counts[chunk] = cnt;
}

// Packed 8-byte double-array records (built by gbpe_trie_upload):
//   x = check (22 bits) | tokenId bits 0-9 << 22,  y = base (22 bits) | tokenId bits 10-19 << 22
// check 0x3FFFFF = empty slot, tokenId 0xFFFFF = none, base 0 = leaf (no children).
__device__ __forceinline__ uint32_t rec_check(uint2 r) { return r.x & 0x3FFFFFu; }
__device__ __forceinline__ uint32_t rec_base(uint2 r) { return r.y & 0x3FFFFFu; }
__device__ __forceinline__ uint32_t rec_tid(uint2 r) { return (r.x >> 22) | ((r.y >> 22) << 10); }
constexpr uint32_t TID_NONE = 0xFFFFFu;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t win_byte(uint4 w, uint32_t o) {
    const uint32_t d = (o & 8u) ? ((o & 4u) ? w.w : w.z) : ((o & 4u) ? w.y : w.x);
    return (d >> ((o & 3u) * 8u)) & 0xFFu;
}

__device__ __forceinline__ uint4 load_win(const uint8_t* __restrict__ in, uint64_t n, uint64_t ab) {
    if (ab + 16 <= n) return *reinterpret_cast<const uint4*>(in + ab);
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;   // the last partial block: byte loads inside [0, n)
    for (uint32_t j = 0; j < 16 && ab + j < n; ++j) {
        const uint32_t v = (uint32_t)in[ab + j] << ((j & 3) * 8);
        if (j < 4) w0 |= v; else if (j < 8) w1 |= v; else if (j < 12) w2 |= v; else w3 |= v;
    }
    return make_uint4(w0, w1, w2, w3);
}

// 64-byte input window (one cache line per refill): 4 x 16 bytes in registers
struct Win64 {
    uint4 q0, q1, q2, q3;
};
__device__ __forceinline__ Win64 load_win64(const uint8_t* __restrict__ in, uint64_t n, uint64_t ab) {
    Win64 w;
    if (ab + 64 <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(in + ab);
        w.q0 = p[0];
        w.q1 = p[1];
        w.q2 = p[2];
        w.q3 = p[3];
    } else {
        w.q0 = load_win(in, n, ab);
        w.q1 = load_win(in, n, ab + 16);
        w.q2 = load_win(in, n, ab + 32);
        w.q3 = load_win(in, n, ab + 48);
    }
    return w;
}
__device__ __forceinline__ uint32_t win64_byte(const Win64& w, uint32_t o) {
    const uint4 q = (o & 32u) ? ((o & 16u) ? w.q3 : w.q2) : ((o & 16u) ? w.q1 : w.q0);
    return win_byte(q, o & 15u);
}

// token vector: slot j of a 16-byte register vector (8 x u16 or 4 x u32), stored whole
template <typename T>
__device__ __forceinline__ void vec_put(uint4& a, uint32_t j, uint32_t tok) {
    if (sizeof(T) == 2) {
        const uint32_t sh = (j & 1u) * 16u, q = (j >> 1) & 3u;
        const uint32_t v = (tok & 0xFFFFu) << sh;
        a.x |= q == 0 ? v : 0u;
        a.y |= q == 1 ? v : 0u;
        a.z |= q == 2 ? v : 0u;
        a.w |= q == 3 ? v : 0u;
    } else {
        const uint32_t q = j & 3u;
        a.x = q == 0 ? tok : a.x;
        a.y = q == 1 ? tok : a.y;
        a.z = q == 2 ? tok : a.z;
        a.w = q == 3 ? tok : a.w;
    }
}

// Production walk.  One lane per chunk (as tokenize.wgsl:88) over the packed
// 8-byte double-array records, as a one-byte-per-trip state machine: every loop
// trip a lane consumes exactly one byte — a token start resolved from the root
// transitions cached in LDS, or one trie transition (the trip's single L2 load);
// a start that leads into a multi-byte path does its first transition in the same
// trip, and a walk that enters a leaf (base == 0) ends its token without the
// probe that would only find the mismatch.  No lane waits on another lane's run
// of raw / one-byte tokens (an inner start loop made the wave's walking lanes
// wait: 4.84 vs 4.29 ms on C3).  Input arrives a 64-byte line per refill: with
// ~65K lanes per XCD walking, 16-byte refills were evicted from the 4 MB L2
// between uses (5.33 vs 4.84 ms).
#ifndef GBPE_WALK_QV
#define GBPE_WALK_QV 4
#endif
constexpr uint32_t WALK_QV = GBPE_WALK_QV;   // token vectors per scratch store burst

template <typename T>
__global__ __launch_bounds__(WALK_TPB) void k_trie_walk_v5(const uint8_t* __restrict__ in, uint64_t n, uint32_t cs,
                                                           const uint2* __restrict__ rec, uint32_t nrec,
                                                           uint32_t root_base, T* __restrict__ scratch,
                                                           uint32_t* __restrict__ counts, uint64_t nchunks) {
    constexpr uint32_t PER = 16 / sizeof(T);
    __shared__ uint2 lut[256];
    {
        const uint32_t t = root_base + threadIdx.x;
        lut[threadIdx.x] = t < nrec ? rec[t] : make_uint2(0x3FFFFFu, 0u);
    }
    __syncthreads();
    const uint64_t chunk = (uint64_t)blockIdx.x * WALK_TPB + threadIdx.x;
    if (chunk >= nchunks) return;
    const uint64_t c0 = chunk * cs;
    const uint32_t ce = (uint32_t)(min(c0 + cs, n) - c0);
    T* out = scratch + c0;
    uint32_t cb = ~0u;
    Win64 w64{};
    uint4 acc = make_uint4(0, 0, 0, 0);
    auto byte_at = [&](uint32_t p) -> uint32_t {
        const uint32_t b = p & ~63u;
        if (b != cb) {
            cb = b;
            w64 = load_win64(in, n, c0 + b);
        }
        return win64_byte(w64, p & 63u);
    };
    // Completed vectors wait in registers and leave WALK_QV at a time, 64
    // contiguous bytes per lane: 3.85 ms against 4.06 for one 16-byte store per
    // vector on C3 (tokens equal).  Wave-wide bursts (every lane stores
    // when one lane's queue is full) measured the same, and at a 2-vector queue
    // slower (4.09 ms).
    uint32_t cnt = 0, nq = 0;
    uint4 q[WALK_QV > 1 ? WALK_QV - 1 : 1];   // q[WALK_QV-1-nq ..]: the nq waiting vectors, oldest first
    auto emit = [&](uint32_t tok) {
        vec_put<T>(acc, cnt % PER, tok);
        if (++cnt % PER == 0) {
            if (nq == WALK_QV - 1) {
#ifndef GBPE_WALK_NOSTORE   // (diagnostic build: the walk without its scratch stores)
                uint4* o = reinterpret_cast<uint4*>(out + cnt) - WALK_QV;
#pragma unroll
                for (uint32_t i = 0; i + 1 < WALK_QV; ++i) o[i] = q[i];
                o[WALK_QV - 1] = acc;
#endif
                nq = 0;
            } else {
                if constexpr (WALK_QV > 1) {
#pragma unroll
                    for (uint32_t i = 0; i + 2 < WALK_QV; ++i) q[i] = q[i + 1];
                    q[WALK_QV - 2] = acc;
                }
                ++nq;
            }
            acc = make_uint4(0, 0, 0, 0);
        }
    };
    auto flush = [&]() {   // the waiting vectors end where the partial vector starts
        if constexpr (WALK_QV > 1) {
            uint4* o = reinterpret_cast<uint4*>(out + (cnt / PER) * PER);
#pragma unroll
            for (uint32_t i = 0; i + 1 < WALK_QV; ++i)
                if (i + nq >= WALK_QV - 1) o[(int)i - (int)WALK_QV + 1] = q[i];
            nq = 0;
        }
    };
    uint32_t pos = 0, wp = 0, lmp = 0, st = 0, base = 0, lmt = TID_NONE, first = 0;
    bool walking = false;
    while (pos < ce) {
        if (!walking) {   // a token start: LDS only
            first = byte_at(pos);
            const uint2 e = lut[first];
            const uint32_t tid = rec_tid(e);
            if (rec_check(e) != 0u || rec_base(e) == 0u || pos + 1 >= ce) {
                // no token starts with this byte (emit it raw, tokenize.wgsl:169-171), a
                // one-byte leaf, or the chunk's last byte
                emit(rec_check(e) == 0u && tid != TID_NONE ? tid : first);
                ++pos;
                continue;
            }
            st = root_base + first;
            base = rec_base(e);
            lmt = tid;
            lmp = pos + 1;
            wp = pos + 1;
            walking = true;
        }
        // one trie transition: the trip's L2 load
        const uint32_t t = base + byte_at(wp);
        const uint2 r = t < nrec ? rec[t] : make_uint2(0x3FFFFFu, 0u);
        bool end = true;
        if (rec_check(r) == st) {
            st = t;
            base = rec_base(r);
            ++wp;
            const uint32_t tid = rec_tid(r);
            if (tid != TID_NONE) {
                lmt = tid;
                lmp = wp;
            }
            end = base == 0u || wp >= ce;
        }
        if (end) {   // the longest match ends: emit it (or the raw first byte), restart after it
            const bool hit = lmt != TID_NONE;
            emit(hit ? lmt : first);
            pos = hit ? lmp : pos + 1;
            walking = false;
        }
    }
    flush();
    if (cnt % PER) *reinterpret_cast<uint4*>(out + (cnt / PER) * PER) = acc;
    counts[chunk] = cnt;
}

#ifdef GBPE_WALK_ALLPOS
// Diagnostic build only ("One wave per chunk, measured"): the
// first half of a wave-per-chunk walk — the longest match from EVERY byte
// position, one lane per position, the workgroup's bytes staged in LDS — so that
// its cost, a lower bound on that design (the greedy path through the per-position
// matches comes on top), is measured against the one-lane-per-chunk walk above.
__global__ __launch_bounds__(WALK_TPB) void k_match_allpos(const uint8_t* __restrict__ in, uint64_t n, uint32_t cs,
                                                           const uint2* __restrict__ rec, uint32_t nrec,
                                                           uint32_t root_base, uint8_t* __restrict__ lens) {
    constexpr uint32_t SPAN = 3 * WALK_TPB;
    __shared__ uint2 lut[256];
    __shared__ uint8_t buf[SPAN];
    {
        const uint32_t t = root_base + threadIdx.x;
        lut[threadIdx.x] = t < nrec ? rec[t] : make_uint2(0x3FFFFFu, 0u);
    }
    const uint64_t p0 = (uint64_t)blockIdx.x * WALK_TPB;
    for (uint32_t i = threadIdx.x; i < SPAN; i += WALK_TPB) buf[i] = p0 + i < n ? in[p0 + i] : 0;
    __syncthreads();
    const uint64_t p = p0 + threadIdx.x;
    if (p >= n) return;
    const uint64_t ce = min((p / cs + 1) * cs, n);
    const uint32_t first = buf[threadIdx.x];
    const uint2 e = lut[first];
    uint32_t len = 1, tok = first;
    if (rec_check(e) == 0u) {
        if (rec_tid(e) != TID_NONE) tok = rec_tid(e);
        uint32_t st = root_base + first, base = rec_base(e);
        uint64_t wp = p + 1;
        while (base != 0u && wp < ce) {
            const uint32_t b = wp - p0 < SPAN ? buf[wp - p0] : in[wp];
            const uint32_t t = base + b;
            const uint2 r = t < nrec ? rec[t] : make_uint2(0x3FFFFFu, 0u);
            if (rec_check(r) != st) break;
            st = t;
            base = rec_base(r);
            ++wp;
            if (rec_tid(r) != TID_NONE) {
                tok = rec_tid(r);
                len = (uint32_t)(wp - p);
            }
        }
    }
    lens[p] = (uint8_t)(min(len, 255u) ^ tok);   // (the token keeps its loads live)
}
#endif

// Chunk tokens → final positions.  A wave moves CPW chunks at once (every
// scratch load of the CPW chunks is issued before the first store: one chunk's
// ~cs/4 tokens alone leave too few bytes in flight to cover the HBM latency);
// token j + 64k of a chunk pass goes to lane j, so every u32 store instruction
// writes 256 contiguous bytes.  Chunks of more than 256 tokens take more passes.
constexpr int CPW = 4;   // chunks per wave
template <typename T>
__global__ __launch_bounds__(256) void k_chunk_compact4(const T* __restrict__ scratch, const uint32_t* __restrict__ counts,
                                                        const uint32_t* __restrict__ local,
                                                        const uint64_t* __restrict__ blocksum, uint64_t nchunks,
                                                        uint32_t cs, uint32_t* __restrict__ out, uint64_t out_cap) {
    __shared__ uint64_t s_off[4 * CPW];
    __shared__ uint32_t s_cnt[4 * CPW];
    const uint64_t c0 = (uint64_t)blockIdx.x * (4 * CPW);
    if (threadIdx.x < 4 * CPW) {
        const uint64_t c = c0 + threadIdx.x;
        s_cnt[threadIdx.x] = c < nchunks ? counts[c] : 0u;
        s_off[threadIdx.x] = c < nchunks ? blocksum[c / SCAN_BLK] + local[c] : 0ull;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t most = 0;
#pragma unroll
    for (int q = 0; q < CPW; ++q) most = max(most, s_cnt[wid * CPW + q]);
    for (uint32_t b0 = 0; b0 < most; b0 += 256) {
        uint32_t v[CPW][4];
#pragma unroll
        for (int q = 0; q < CPW; ++q) {
            const uint32_t cnt = s_cnt[wid * CPW + q];
            const T* src = scratch + (c0 + wid * CPW + q) * (uint64_t)cs;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = b0 + lane + 64u * k;
                v[q][k] = j < cnt ? (uint32_t)src[j] : 0u;
            }
        }
#pragma unroll
        for (int q = 0; q < CPW; ++q) {
            const uint32_t cnt = s_cnt[wid * CPW + q];
            const uint64_t off = s_off[wid * CPW + q];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = b0 + lane + 64u * k;
                if (j < cnt && off + j < out_cap) out[off + j] = v[q][k];
            }
        }
    }
}

}  // namespace

struct gbpe_trie {
    gbpe_ctx* ctx = nullptr;
    uint4* rec = nullptr;      // double-array records {check, base, tokenId, 0}
    uint2* rec2 = nullptr;     // packed 8-byte records (pack_rec); null when ids / states do not fit
    uint32_t root_base = 0;    // base of the root state
    uint32_t nrec = 0;
    uint4* root = nullptr;     // 256 root transitions {state, base, tokenId, present}
    uint32_t max_token_len = 0;
    uint32_t max_token_id = 0;
    uint32_t n_nodes = 0, n_edges = 0;
};

extern "C" int gbpe_trie_upload(gbpe_ctx* ctx, const uint32_t* nodes, uint32_t n_nodes, const uint32_t* edges,
                                uint32_t n_edges, gbpe_trie** out) {
    if (!ctx || !out || !nodes || n_nodes == 0 || (!edges && n_edges))
        return gbpe_set_error(ctx, GBPE_E_INVALID, "trie upload: bad arguments");
    *out = nullptr;
    // ── compile the BFS trie into a double array ──
    // state ids: root = 0 (never a transition target); every other node gets
    // slot base(parent) + byte.
    std::vector<uint32_t> state(n_nodes, INV), depth(n_nodes, 0);
    std::vector<uint4> rec(1, make_uint4(INV, 0, INV, 0));  // slot 0 reserved for the root
    std::vector<uint8_t> used(1, 1);
    uint32_t first_free = 1;
    std::vector<uint32_t> queue;
    queue.reserve(n_nodes);
    queue.push_back(0);
    state[0] = 0;
    uint32_t max_len = 0, max_tid = 0, root_base = 0;
    auto ensure = [&](uint64_t sz) {
        if (sz > rec.size()) {
            rec.resize(sz, make_uint4(INV, 0, INV, 0));
            used.resize(sz, 0);
        }
    };
    std::vector<uint4> root(256, make_uint4(0, 0, INV, 0));
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const uint32_t u = queue[qi];
        const uint32_t fc = nodes[3 * (uint64_t)u], nc = nodes[3 * (uint64_t)u + 1] & 0xFFFFu;
        if (nc && (uint64_t)fc + nc > n_edges)
            return gbpe_set_error(ctx, GBPE_E_INVALID, "trie upload: node %u edges out of range", u);
        uint32_t prev = 0;
        for (uint32_t k = 0; k < nc; ++k) {
            uint32_t c = edges[2 * ((uint64_t)fc + k)] & 0xFFu;
            if (k && c <= prev)
                return gbpe_set_error(ctx, GBPE_E_INVALID, "trie upload: children of node %u not sorted/unique", u);
            prev = c;
        }
        if (nc == 0) continue;
        const uint32_t cmin = edges[2 * (uint64_t)fc] & 0xFFu;
        // first-fit base search
        uint32_t b = first_free > cmin ? first_free - cmin : 1;
        if (b < 1) b = 1;
        for (;; ++b) {
            ensure((uint64_t)b + 256);
            bool ok = true;
            for (uint32_t k = 0; k < nc && ok; ++k) ok = !used[b + (edges[2 * ((uint64_t)fc + k)] & 0xFFu)];
            if (ok) break;
        }
        const uint32_t su = state[u];
        if (u != 0) rec[su].y = b;
        else root_base = b;
        for (uint32_t k = 0; k < nc; ++k) {
            const uint32_t c = edges[2 * ((uint64_t)fc + k)] & 0xFFu;
            const uint32_t v = edges[2 * ((uint64_t)fc + k) + 1];
            if (v >= n_nodes || v == 0) return gbpe_set_error(ctx, GBPE_E_INVALID, "trie upload: bad edge target %u", v);
            if (state[v] != INV) return gbpe_set_error(ctx, GBPE_E_INVALID, "trie upload: node %u reached twice (not a tree)", v);
            const uint32_t t = b + c;
            used[t] = 1;
            state[v] = t;
            depth[v] = depth[u] + 1;
            const uint32_t tid = nodes[3 * (uint64_t)v + 2];
            rec[t] = make_uint4(su, 0, tid, 0);
            if (tid != INV) {
                max_len = std::max(max_len, depth[v]);
                max_tid = std::max(max_tid, tid);
            }
            queue.push_back(v);
            if (u == 0) root[c] = make_uint4(t, 0, tid, 1);
        }
        while (first_free < used.size() && used[first_free]) ++first_free;
    }
    // root LUT entries need their child's base (filled after the BFS)
    for (int c = 0; c < 256; ++c)
        if (root[c].w) root[c].y = rec[root[c].x].y;
    auto* tr = new (std::nothrow) gbpe_trie();
    if (!tr) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    tr->ctx = ctx;
    tr->nrec = (uint32_t)rec.size();
    tr->max_token_len = max_len;
    tr->max_token_id = max_tid;
    tr->n_nodes = n_nodes;
    tr->n_edges = n_edges;
    tr->root_base = root_base;
    hipError_t e = dev_malloc(ctx, &tr->rec, rec.size() * sizeof(uint4));
    if (e == hipSuccess) e = dev_malloc(ctx, &tr->root, 256 * sizeof(uint4));
    if (e == hipSuccess) e = hipMemcpy(tr->rec, rec.data(), rec.size() * sizeof(uint4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(tr->root, root.data(), 256 * sizeof(uint4), hipMemcpyHostToDevice);
    // packed records: check (22 bits) | tid low 10 << 22, base (22 bits) | tid high 10 << 22
    const bool packable = rec.size() + 256 < 0x3FFFFFu && max_tid < 0xFFFFFu;
    if (e == hipSuccess && packable) {
        std::vector<uint2> r2(rec.size() + 256);
        for (size_t i = 0; i < r2.size(); ++i) {
            const uint4 q = i < rec.size() ? rec[i] : make_uint4(INV, 0, INV, 0);
            const uint32_t chk = q.x == INV ? 0x3FFFFFu : q.x;
            const uint32_t tid = q.z == INV ? 0xFFFFFu : q.z;
            r2[i] = make_uint2(chk | ((tid & 0x3FFu) << 22), (q.y & 0x3FFFFFu) | ((tid >> 10) << 22));
        }
        e = dev_malloc(ctx, &tr->rec2, r2.size() * sizeof(uint2));
        if (e == hipSuccess) e = hipMemcpy(tr->rec2, r2.data(), r2.size() * sizeof(uint2), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        gbpe_trie_free(tr);
        return gbpe_set_error(ctx, GBPE_E_DEVICE, "trie upload failed: %s", hipGetErrorString(e));
    }
    *out = tr;
    return GBPE_OK;
}

extern "C" int gbpe_trie_info(const gbpe_trie* tr, uint32_t* n_records, uint32_t* max_token_len, uint32_t* max_token_id) {
    if (!tr) return GBPE_E_INVALID;
    if (n_records) *n_records = tr->nrec;
    if (max_token_len) *max_token_len = tr->max_token_len;
    if (max_token_id) *max_token_id = tr->max_token_id;
    return GBPE_OK;
}

extern "C" void gbpe_trie_free(gbpe_trie* tr) {
    if (!tr) return;
    hipFree(tr->rec);
    hipFree(tr->rec2);
    hipFree(tr->root);
    delete tr;
}

namespace {

int grow(gbpe_ctx* ctx, void** p, uint64_t* have, uint64_t need) {
    if (*have >= need) return GBPE_OK;
    if (*p) {
        hipStreamSynchronize(ctx->stream);
        hipFree(*p);
        *p = nullptr;
        *have = 0;
    }
    const uint64_t sz = need + need / 2;   // 1.5x amortised growth (tokenizer.js:125-128)
    GBPE_HIP(ctx, dev_malloc(ctx, p, sz));
    *have = sz;
    return GBPE_OK;
}

uint32_t effective_cs(const gbpe_trie* tr, uint32_t cs) {
    if (cs) return cs;
    // tokenizer.js:67-68 adaptive chunk
    const uint32_t a = tr->max_token_len * 8u;
    return std::max<uint32_t>(512u, std::min<uint32_t>(2048u, a));
}

// runs the three encode kernels on device buffers; *total_dev receives the count
int encode_device_impl(gbpe_ctx* ctx, gbpe_trie* tr, const uint8_t* d_in, uint64_t n, uint32_t cs, uint32_t* d_out,
                       uint64_t out_cap, uint64_t* n_out) {
    hipStream_t s = ctx->stream;
    const uint64_t nchunks = gbpe_div_up(n, cs);
    const bool narrow = tr->max_token_id < 65536u;   // raw-byte fallbacks are < 256
    const uint64_t esz = narrow ? 2 : 4;
    const uint64_t nblk = gbpe_div_up(nchunks, SCAN_BLK);
    int rc = grow(ctx, &ctx->enc_scratch, &ctx->enc_scratch_bytes, nchunks * cs * esz + 16);
    if (rc == GBPE_OK)
        rc = grow(ctx, &ctx->enc_counts, &ctx->enc_counts_bytes, nchunks * 8 + nblk * 8 + 64);
    if (rc != GBPE_OK) return rc;
    uint32_t* counts = (uint32_t*)ctx->enc_counts;
    uint32_t* local = counts + nchunks;
    uint64_t* blocksum = (uint64_t*)(((uintptr_t)(local + nchunks) + 15) & ~(uintptr_t)15);
    uint64_t* d_total = blocksum + nblk + 1;
    const uint32_t gw = (uint32_t)gbpe_div_up(nchunks, WALK_TPB);
#ifdef GBPE_WALK_ALLPOS
    if (tr->rec2 && out_cap * 4 >= n) {   // (diagnostic build: d_out is free scratch until the compaction)
        GBPE_HIP(ctx, hipEventRecord(ctx->ev[0], s));
        hipLaunchKernelGGL(k_match_allpos, dim3((uint32_t)gbpe_div_up(n, WALK_TPB)), dim3(WALK_TPB), 0, s, d_in, n, cs,
                           tr->rec2, tr->nrec + 256, tr->root_base, (uint8_t*)d_out);
        GBPE_LAUNCH_CHECK(ctx);
        GBPE_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        GBPE_HIP(ctx, hipEventSynchronize(ctx->ev[1]));
        float ms = 0;
        hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
        fprintf(stderr, "[allpos] %.3f ms\n", ms);
    }
#endif
    GBPE_HIP(ctx, hipEventRecord(ctx->ev[0], s));
    // the packed-record state-machine walk when the trie packs and chunks are whole
    // 16-byte token vectors (cs % 8 == 0: every adaptive chunk size); otherwise the
    // plain per-token walk over 16-byte records
    const bool packed = (cs % 8u) == 0u && tr->rec2;
    const uint32_t nrec2 = tr->nrec + 256;
    if (packed && narrow)
        hipLaunchKernelGGL(k_trie_walk_v5<uint16_t>, dim3(gw), dim3(WALK_TPB), 0, s, d_in, n, cs, tr->rec2, nrec2,
                           tr->root_base, (uint16_t*)ctx->enc_scratch, counts, nchunks);
    else if (packed)
        hipLaunchKernelGGL(k_trie_walk_v5<uint32_t>, dim3(gw), dim3(WALK_TPB), 0, s, d_in, n, cs, tr->rec2, nrec2,
                           tr->root_base, (uint32_t*)ctx->enc_scratch, counts, nchunks);
    else if (narrow)
        hipLaunchKernelGGL(k_trie_walk<uint16_t>, dim3(gw), dim3(WALK_TPB), 0, s, d_in, n, cs, tr->rec, tr->nrec,
                           tr->root, (uint16_t*)ctx->enc_scratch, counts, nchunks);
    else
        hipLaunchKernelGGL(k_trie_walk<uint32_t>, dim3(gw), dim3(WALK_TPB), 0, s, d_in, n, cs, tr->rec, tr->nrec,
                           tr->root, (uint32_t*)ctx->enc_scratch, counts, nchunks);
    GBPE_LAUNCH_CHECK(ctx);
    GBPE_HIP(ctx, hipEventRecord(ctx->ev[1], s));
    hipLaunchKernelGGL(k_chunk_scan1, dim3((uint32_t)nblk), dim3(SCAN_TPB), 0, s, (const uint32_t*)counts, nchunks, local,
                       blocksum);
    hipLaunchKernelGGL(k_chunk_scan2, dim3(1), dim3(SCAN_TPB), 0, s, blocksum, nblk, d_total);
    GBPE_LAUNCH_CHECK(ctx);
    GBPE_HIP(ctx, hipEventRecord(ctx->ev[2], s));
    const uint32_t gc4 = (uint32_t)gbpe_div_up(nchunks, 4 * CPW);
    if (narrow)
        hipLaunchKernelGGL(k_chunk_compact4<uint16_t>, dim3(gc4), dim3(256), 0, s, (const uint16_t*)ctx->enc_scratch,
                           (const uint32_t*)counts, (const uint32_t*)local, (const uint64_t*)blocksum, nchunks, cs, d_out,
                           out_cap);
    else
        hipLaunchKernelGGL(k_chunk_compact4<uint32_t>, dim3(gc4), dim3(256), 0, s, (const uint32_t*)ctx->enc_scratch,
                           (const uint32_t*)counts, (const uint32_t*)local, (const uint64_t*)blocksum, nchunks, cs, d_out,
                           out_cap);
    GBPE_LAUNCH_CHECK(ctx);
    GBPE_HIP(ctx, hipEventRecord(ctx->ev[3], s));
    GBPE_HIP(ctx, hipMemcpyAsync(ctx->enc_host_total, d_total, 8, hipMemcpyDeviceToHost, s));
    GBPE_HIP(ctx, hipStreamSynchronize(s));
    float a = 0, b = 0, c = 0;
    hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]);
    hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[2]);
    hipEventElapsedTime(&c, ctx->ev[2], ctx->ev[3]);
    ctx->enc_ms[0] = a;
    ctx->enc_ms[1] = b;
    ctx->enc_ms[2] = c;
    uint64_t total;
    memcpy(&total, ctx->enc_host_total, 8);
    *n_out = total;
    if (total > out_cap) return gbpe_set_error(ctx, GBPE_E_CAPACITY, "encode: output needs %llu tokens", (unsigned long long)total);
    return GBPE_OK;
}

}  // namespace

extern "C" int gbpe_encode_device(gbpe_ctx* ctx, gbpe_trie* tr, const void* d_bytes, uint64_t n, uint32_t chunk_size,
                                  void* d_out, uint64_t out_cap, uint64_t* n_out) {
    if (!ctx || !tr || !n_out || (n && (!d_bytes || !d_out))) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    if ((uintptr_t)d_bytes & 3u) return gbpe_set_error(ctx, GBPE_E_INVALID, "d_bytes must be 4-byte aligned");
    *n_out = 0;
    if (n == 0) return GBPE_OK;
    return encode_device_impl(ctx, tr, (const uint8_t*)d_bytes, n, effective_cs(tr, chunk_size), (uint32_t*)d_out,
                              out_cap, n_out);
}

// Host buffers in and out (tokenizer.js:213-335 incl. the readback).  Inputs
// larger than one slice run as a pipeline of chunk-aligned slices: while the
// device encodes slice i+1 (after its upload), a second host thread copies slice
// i's tokens back, so uploads, kernels and downloads overlap.  Slices start at
// multiples of 64 * chunk size, so every chunk — and every token — is the one a
// single pass produces.
extern "C" int gbpe_encode(gbpe_ctx* ctx, gbpe_trie* tr, const uint8_t* bytes, uint64_t n, uint32_t chunk_size,
                           uint32_t* out, uint64_t out_cap, uint64_t* n_out) {
    if (!ctx || !tr || !n_out || (n && !bytes)) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *n_out = 0;
    if (n == 0) return GBPE_OK;   // tokenizer.js:175
    const uint32_t cs = effective_cs(tr, chunk_size);
    int rc = grow(ctx, &ctx->enc_in, &ctx->enc_in_bytes, gbpe_div_up(n, 4) * 4 + 16);
    if (rc == GBPE_OK) rc = grow(ctx, &ctx->enc_out, &ctx->enc_out_bytes, n * 4 + 16);   // <= 1 token per byte
    if (rc != GBPE_OK) return rc;
    const uint64_t unit = (uint64_t)cs * 64;
    // (test override: many slices on small inputs)
    const uint64_t want = (uint64_t)std::max<long>(1, gbpe_debug_knob("encode_slice", (long)kEncSlice));
    const uint64_t slice = std::max<uint64_t>(unit, (want / unit) * unit);
    uint8_t* d_in = (uint8_t*)ctx->enc_in;
    uint32_t* d_out = (uint32_t*)ctx->enc_out;
    if (n <= slice) {
        GBPE_HIP(ctx, hipMemcpyAsync(d_in, bytes, n, hipMemcpyHostToDevice, ctx->stream));
        uint64_t total = 0;
        rc = encode_device_impl(ctx, tr, d_in, n, cs, d_out, n, &total);
        *n_out = total;
        if (rc != GBPE_OK) return rc;
        if (total > out_cap)
            return gbpe_set_error(ctx, GBPE_E_CAPACITY, "encode: output needs %llu tokens", (unsigned long long)total);
        if (total) {
            GBPE_HIP(ctx, hipMemcpyAsync(out, d_out, total * 4, hipMemcpyDeviceToHost, ctx->stream));
            GBPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        }
        return GBPE_OK;
    }
    if (!ctx->copy_stream) GBPE_HIP(ctx, hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    struct Part {
        uint64_t off, cnt;
    };
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Part> q;
    bool finished = false;
    hipError_t copy_err = hipSuccess;
    hipStream_t so = ctx->copy_stream;
    const int dev = ctx->device;
    std::thread drain([&]() {
        hipSetDevice(dev);
        for (;;) {
            Part p;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return finished || !q.empty(); });
                if (q.empty()) return;
                p = q.front();
                q.pop_front();
            }
            if (copy_err != hipSuccess) continue;
            hipError_t e = hipMemcpyAsync(out + p.off, d_out + p.off, p.cnt * 4, hipMemcpyDeviceToHost, so);
            if (e == hipSuccess) e = hipStreamSynchronize(so);
            if (e != hipSuccess) copy_err = e;
        }
    });
    uint64_t total = 0;
    for (uint64_t s0 = 0; s0 < n && rc == GBPE_OK; s0 += slice) {
        const uint64_t len = std::min(slice, n - s0);
        hipError_t e = hipMemcpyAsync(d_in + s0, bytes + s0, len, hipMemcpyHostToDevice, ctx->stream);
        if (e != hipSuccess) {
            rc = gbpe_set_error(ctx, GBPE_E_DEVICE, "encode upload failed: %s", hipGetErrorString(e));
            break;
        }
        uint64_t t = 0;
        rc = encode_device_impl(ctx, tr, d_in + s0, len, cs, d_out + total, n - total, &t);   // (synchronises)
        if (rc != GBPE_OK) break;
        if (t && total + t <= out_cap) {
            std::lock_guard<std::mutex> g(mu);
            q.push_back(Part{total, t});
            cv.notify_one();
        }
        total += t;
    }
    {
        std::lock_guard<std::mutex> g(mu);
        finished = true;
        cv.notify_one();
    }
    drain.join();
    *n_out = total;
    if (rc != GBPE_OK) return rc;
    if (copy_err != hipSuccess) return gbpe_set_error(ctx, GBPE_E_DEVICE, "encode readback failed: %s", hipGetErrorString(copy_err));
    if (total > out_cap) return gbpe_set_error(ctx, GBPE_E_CAPACITY, "encode: output needs %llu tokens", (unsigned long long)total);
    return GBPE_OK;
}

extern "C" int gbpe_encode_last_timing(gbpe_ctx* ctx, double* ms_walk, double* ms_scan, double* ms_compact) {
    if (!ctx) return GBPE_E_INVALID;
    if (ms_walk) *ms_walk = ctx->enc_ms[0];
    if (ms_scan) *ms_scan = ctx->enc_ms[1];
    if (ms_compact) *ms_compact = ctx->enc_ms[2];
    return GBPE_OK;
}
