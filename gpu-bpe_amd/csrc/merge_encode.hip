// Merge-rank BPE encode on MI355X: TokenizerManager.encode
// (src/bpe/tokenizer/tokenizer-manager.js:13-61), the UI tab's encoder.
//
// The reference applies every learned merge in order to the whole byte string
// (one left-to-right pass per merge).  Two facts make that parallel and exact:
//   * a merge's new pairs involve its new token, whose id is only used by
//     later merges — so applying ranks in order equals repeatedly applying the
//     lowest-rank adjacent pair (all its occurrences, left to right);
//   * a token can only ever span the boundary between bytes (u, v) if some
//     merge (a, b) has last(a) = u and first(b) = v.  Every other boundary is a
//     cut no merge crosses, so the text splits into independent segments.
// A merge whose operand is created by a LATER merge (or never) never fires in
// the reference; such merges are dropped on upload, as are repeated pairs
// (the first rank wins, tokenizer-manager.js:30-33).
//
// k_me_walk: one lane per 4096-byte chunk; it owns the segments that START in
// its chunk and BPE-encodes each in place (rank lookups in an L2-resident
// open-addressing table).  Chunk counts → scan.h two-level scan → k_me_compact.
// A segment longer than ME_LONG bytes (CJK paragraphs, base64, minified code:
// no cut for a long stretch) would cost its lane one full pass per rank
// applied; it is encoded with a rank-ordered heap over a linked list instead
// (me_heap: O(len log len), same order: lowest rank first, leftmost first),
// in an arena k_me_long sized and laid out beforehand.

#include "common.h"
#include "scan.h"

#include <vector>

namespace {

constexpr int ME_TPB = 64;
constexpr uint32_t ME_CS = 4096;      // bytes per chunk (a lane's range of segment starts)
constexpr uint32_t ME_NONE = 0xFFFFFFFFu;
constexpr uint32_t ME_LONG = 1024;                  // longer segments take the heap path
constexpr uint32_t ME_LSLOT = ME_CS / ME_LONG + 1;  // long segments that can start in one chunk
constexpr uint32_t ME_DEAD = 0xFFFFFFFFu;

struct MeArena {   // per long segment at offset `off` (bytes of all long segments before it)
    uint32_t* tok;       // [off, off + len)
    uint32_t* nxt;
    uint32_t* prv;
    uint64_t* heap;      // [3 off, 3 (off + len)): initial pairs + two per merge
    const uint64_t* slot;   // per chunk: ME_LSLOT offsets of the long segments starting in it
};

struct MeTable {
    const uint4* slots;   // {pid, rank, new id, 0}; pid 0 = empty ((0,0) never merges: token 0 never pairs)
    uint32_t mask;
    const uint32_t* cross;   // 65536-bit: (u << 8 | v) set iff some merge joins a token ending in u to one starting with v
};

__device__ __forceinline__ uint4 me_find(const MeTable& t, uint32_t pid) {
    uint32_t h = gbpe_fmix32(pid) & t.mask;
    for (uint32_t p = 0; p <= t.mask; ++p) {
        const uint32_t idx = (h + ((p * (p + 1)) >> 1)) & t.mask;
        const uint4 e = t.slots[idx];
        if (e.x == pid) return e;
        if (e.x == 0u) break;
    }
    return make_uint4(0u, ME_NONE, 0u, 0u);
}

__device__ __forceinline__ bool me_cut(const uint8_t* __restrict__ in, const MeTable& t, uint64_t i) {
    if (i == 0) return true;
    const uint32_t k = ((uint32_t)in[i - 1] << 8) | in[i];
    return ((t.cross[k >> 5] >> (k & 31u)) & 1u) == 0u;
}

// the long segments (> ME_LONG bytes) starting in each chunk: arena offsets
__global__ __launch_bounds__(ME_TPB) void k_me_long(const uint8_t* __restrict__ in, uint64_t n, MeTable t,
                                                    unsigned long long* __restrict__ total, uint64_t* __restrict__ slot,
                                                    uint64_t nchunks) {
    const uint64_t c = (uint64_t)blockIdx.x * ME_TPB + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t lo = c * ME_CS, hi = min(lo + ME_CS, n);
    uint64_t s = lo;
    while (s < hi && !me_cut(in, t, s)) ++s;
    uint32_t k = 0;
    while (s < hi) {
        uint64_t z = s + 1;
        while (z < n && !me_cut(in, t, z)) ++z;
        if (z - s > ME_LONG) slot[c * ME_LSLOT + k++] = atomicAdd(total, (unsigned long long)(z - s));
        s = z;
    }
}

// one long segment on one lane: a min-heap of (rank << 32 | position) over the
// adjacent pairs of a doubly linked token list.  Popping the lowest rank, then
// the leftmost position, applies every merge in rank order and each rank's
// occurrences left to right, as the reference's one pass per merge does: a
// merge's new pairs hold its new token, which only later ranks use.  Stale
// entries (the pair at that position changed) are skipped on pop.
__device__ uint32_t me_heap(const uint8_t* __restrict__ in, uint32_t len, const MeTable& t, uint32_t* __restrict__ tk,
                            uint32_t* __restrict__ nx, uint32_t* __restrict__ pv, uint64_t* __restrict__ hp,
                            uint32_t* __restrict__ out) {
    for (uint32_t i = 0; i < len; ++i) {
        tk[i] = in[i];
        nx[i] = i + 1;
        pv[i] = i ? i - 1 : ME_NONE;
    }
    uint32_t h = 0;
    auto push = [&](uint64_t key) {
        uint32_t i = h++;
        while (i) {
            const uint32_t p = (i - 1) >> 1;
            if (hp[p] <= key) break;
            hp[i] = hp[p];
            i = p;
        }
        hp[i] = key;
    };
    auto rank_at = [&](uint32_t i, uint32_t j) -> uint4 { return me_find(t, (tk[i] << 16) | tk[j]); };
    for (uint32_t i = 0; i + 1 < len; ++i) {
        const uint4 e = rank_at(i, i + 1);
        if (e.y != ME_NONE) push(((uint64_t)e.y << 32) | i);
    }
    while (h) {
        const uint64_t key = hp[0];
        const uint64_t last = hp[--h];
        if (h) {   // sift the last entry down from the root
            uint32_t i = 0;
            for (;;) {
                uint32_t c = 2 * i + 1;
                if (c >= h) break;
                if (c + 1 < h && hp[c + 1] < hp[c]) ++c;
                if (last <= hp[c]) break;
                hp[i] = hp[c];
                i = c;
            }
            hp[i] = last;
        }
        const uint32_t r = (uint32_t)(key >> 32), i = (uint32_t)key;
        if (tk[i] == ME_DEAD) continue;
        const uint32_t j = nx[i];
        if (j >= len) continue;
        const uint4 e = rank_at(i, j);
        if (e.y != r) continue;   // stale: the pair at i changed
        tk[i] = e.z;
        tk[j] = ME_DEAD;
        const uint32_t q = nx[j];
        nx[i] = q;
        if (q < len) pv[q] = i;
        const uint32_t p = pv[i];
        if (p != ME_NONE) {
            const uint4 ep = rank_at(p, i);
            if (ep.y != ME_NONE) push(((uint64_t)ep.y << 32) | p);
        }
        if (q < len) {
            const uint4 eq = rank_at(i, q);
            if (eq.y != ME_NONE) push(((uint64_t)eq.y << 32) | i);
        }
    }
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < len; i = nx[i]) out[cnt++] = tk[i];   // position 0 is never merged away
    return cnt;
}

__global__ __launch_bounds__(ME_TPB) void k_me_walk(const uint8_t* __restrict__ in, uint64_t n, MeTable t,
                                                    uint32_t* __restrict__ scratch, uint32_t* __restrict__ counts,
                                                    uint64_t* __restrict__ base, uint64_t nchunks, MeArena ar) {
    const uint64_t c = (uint64_t)blockIdx.x * ME_TPB + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t lo = c * ME_CS, hi = min(lo + ME_CS, n);
    uint64_t s = lo;
    while (s < hi && !me_cut(in, t, s)) ++s;   // first segment start in the chunk
    base[c] = s;
    const uint64_t b0 = s;   // this chunk's tokens go to scratch[b0 ...]: never past the bytes consumed
    uint32_t written = 0, nlong = 0;
    while (s < hi) {
        uint64_t z = s + 1;
        while (z < n && !me_cut(in, t, z)) ++z;   // the segment [s, z) may run past hi
        uint32_t* tok = scratch + b0 + written;
        uint32_t len = (uint32_t)(z - s);
        if (len > ME_LONG) {
            const uint64_t off = ar.slot[c * ME_LSLOT + nlong++];
            written += me_heap(in + s, len, t, ar.tok + off, ar.nxt + off, ar.prv + off, ar.heap + 3 * off, tok);
            s = z;
            continue;
        }
        for (uint32_t j = 0; j < len; ++j) tok[j] = in[s + j];
        while (len >= 2) {
            uint32_t best = ME_NONE, bpid = 0, bnew = 0;
            for (uint32_t j = 0; j + 1 < len; ++j) {
                const uint32_t pid = (tok[j] << 16) | tok[j + 1];
                const uint4 e = me_find(t, pid);
                if (e.y < best) { best = e.y; bpid = pid; bnew = e.z; }
            }
            if (best == ME_NONE) break;
            uint32_t w = 0, j = 0;   // this rank, every occurrence, left to right
            while (j < len) {
                if (j + 1 < len && ((tok[j] << 16) | tok[j + 1]) == bpid) {
                    tok[w++] = bnew;
                    j += 2;
                } else {
                    tok[w++] = tok[j++];
                }
            }
            len = w;
        }
        written += len;
        s = z;
    }
    counts[c] = written;
}

__global__ __launch_bounds__(256) void k_me_compact(const uint32_t* __restrict__ scratch,
                                                    const uint32_t* __restrict__ counts,
                                                    const uint64_t* __restrict__ base, const uint32_t* __restrict__ local,
                                                    const uint64_t* __restrict__ blocksum, uint64_t nchunks,
                                                    uint32_t* __restrict__ out, uint64_t out_cap) {
    const uint64_t chunk = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (chunk >= nchunks) return;
    const int lane = threadIdx.x & 63;
    const uint64_t off = blocksum[chunk / SCAN_BLK] + local[chunk];
    const uint32_t cnt = counts[chunk];
    const uint32_t* src = scratch + base[chunk];
    for (uint32_t j = lane; j < cnt; j += 64) {
        const uint64_t d = off + j;
        if (d < out_cap) out[d] = src[j];
    }
}

}  // namespace

struct gbpe_bpe {
    gbpe_ctx* ctx = nullptr;
    uint4* slots = nullptr;
    uint32_t mask = 0;
    uint32_t* cross = nullptr;
    uint32_t n_live = 0;
};

extern "C" int gbpe_bpe_upload(gbpe_ctx* ctx, const uint32_t* merges, uint32_t n_merges, gbpe_bpe** out) {
    if (!ctx || !out || (n_merges && !merges)) return gbpe_set_error(ctx, GBPE_E_INVALID, "bpe upload: bad arguments");
    *out = nullptr;
    // live merges: both operands exist (bytes, or created by an earlier merge), first rank of a pair
    std::vector<int64_t> created(1u << 16, -1);
    std::vector<uint8_t> first(1u << 16, 0), last(1u << 16, 0);
    for (uint32_t b = 0; b < 256; ++b) { created[b] = -1; first[b] = last[b] = (uint8_t)b; }
    std::vector<uint8_t> exists(1u << 16, 0);
    for (uint32_t b = 0; b < 256; ++b) exists[b] = 1;
    uint32_t slots = 16;
    while (slots < 2u * n_merges + 16) slots <<= 1;
    std::vector<uint4> tab(slots, make_uint4(0, 0, 0, 0));
    std::vector<uint32_t> cross(65536 / 32, 0);
    uint32_t live = 0;
    for (uint32_t r = 0; r < n_merges; ++r) {
        const uint32_t a = merges[3 * (uint64_t)r], b = merges[3 * (uint64_t)r + 1], id = merges[3 * (uint64_t)r + 2];
        if (a > 0xFFFFu || b > 0xFFFFu || id > 0xFFFFu)
            return gbpe_set_error(ctx, GBPE_E_INVALID, "bpe upload: merge %u has an id above 0xFFFF", r);
        if (!exists[a] || !exists[b]) continue;   // an operand that does not exist yet: never fires
        const uint32_t pid = (a << 16) | b;
        if (pid == 0) continue;
        uint32_t h = 0;
        {   // same hash / probing as the device
            uint32_t x = pid;
            x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
            h = x & (slots - 1);
        }
        bool dup = false;
        for (uint32_t p = 0; p < slots; ++p) {
            const uint32_t idx = (h + ((p * (p + 1)) >> 1)) & (slots - 1);
            if (tab[idx].x == pid) { dup = true; break; }
            if (tab[idx].x == 0) { tab[idx] = make_uint4(pid, r, id, 0); break; }
        }
        if (dup) continue;   // the first rank of a pair wins (tokenizer-manager.js:30-33)
        ++live;
        const uint32_t k = ((uint32_t)last[a] << 8) | first[b];
        cross[k >> 5] |= 1u << (k & 31u);
        if (!exists[id]) {
            exists[id] = 1;
            first[id] = first[a];
            last[id] = last[b];
        }
    }
    auto* bp = new (std::nothrow) gbpe_bpe();
    if (!bp) return gbpe_set_error(ctx, GBPE_E_OOM, "host allocation failed");
    bp->ctx = ctx;
    bp->mask = slots - 1;
    bp->n_live = live;
    hipError_t e = dev_malloc(ctx, &bp->slots, slots * sizeof(uint4));
    if (e == hipSuccess) e = dev_malloc(ctx, &bp->cross, cross.size() * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpy(bp->slots, tab.data(), slots * sizeof(uint4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(bp->cross, cross.data(), cross.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        hipFree(bp->slots);
        hipFree(bp->cross);
        delete bp;
        return gbpe_set_error(ctx, GBPE_E_DEVICE, "bpe upload failed: %s", hipGetErrorString(e));
    }
    *out = bp;
    return GBPE_OK;
}

extern "C" void gbpe_bpe_free(gbpe_bpe* bp) {
    if (!bp) return;
    hipFree(bp->slots);
    hipFree(bp->cross);
    delete bp;
}

extern "C" int gbpe_bpe_encode(gbpe_ctx* ctx, gbpe_bpe* bp, const uint8_t* bytes, uint64_t n, uint32_t* out,
                               uint64_t out_cap, uint64_t* n_out) {
    if (!ctx || !bp || !n_out || (n && !bytes)) return gbpe_set_error(ctx, GBPE_E_INVALID, "null argument");
    *n_out = 0;
    if (n == 0) return GBPE_OK;
    hipStream_t s = ctx->stream;
    const uint64_t nchunks = gbpe_div_up(n, ME_CS);
    const uint64_t nblk = gbpe_div_up(nchunks, SCAN_BLK);
    // device buffers: input, scratch tokens (<= 1 per byte), counts, bases, scan state, output
    const uint64_t need = n + 16 + 4 * n + 4 * nchunks + 8 * nchunks + 4 * nchunks + 8 * (nblk + 2) + 4 * n + 64;
    uint8_t* d = nullptr;
    GBPE_HIP(ctx, dev_malloc(ctx, &d, need));
    uint8_t* d_in = d;
    uint32_t* scratch = (uint32_t*)(((uintptr_t)(d + n + 16) + 15) & ~(uintptr_t)15);
    uint32_t* counts = scratch + n;
    uint64_t* base = (uint64_t*)(((uintptr_t)(counts + nchunks) + 15) & ~(uintptr_t)15);
    uint32_t* local = (uint32_t*)(base + nchunks);
    uint64_t* blocksum = (uint64_t*)(((uintptr_t)(local + nchunks) + 15) & ~(uintptr_t)15);
    uint64_t* total = blocksum + nblk + 1;
    uint32_t* d_out = (uint32_t*)(((uintptr_t)(total + 1) + 15) & ~(uintptr_t)15);
    hipError_t e = hipMemcpyAsync(d_in, bytes, n, hipMemcpyHostToDevice, s);
    MeTable t{bp->slots, bp->mask, bp->cross};
    // long segments: their total length sizes the heap arena (none: no arena)
    MeArena ar{};
    uint8_t* da = nullptr;
    uint64_t* slot = nullptr;
    unsigned long long* d_long = nullptr;
    unsigned long long long_total = 0;
    if (e == hipSuccess) e = dev_malloc(ctx, &slot, nchunks * ME_LSLOT * sizeof(uint64_t) + 16);
    if (e == hipSuccess) {
        d_long = (unsigned long long*)(slot + nchunks * ME_LSLOT);
        e = hipMemsetAsync(d_long, 0, 8, s);
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_me_long, dim3((uint32_t)gbpe_div_up(nchunks, ME_TPB)), dim3(ME_TPB), 0, s, d_in, n, t, d_long,
                           slot, nchunks);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&long_total, d_long, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess && long_total) {
        e = dev_malloc(ctx, &da, long_total * (3 * sizeof(uint32_t) + 3 * sizeof(uint64_t)) + 64);
        if (e == hipSuccess) {
            ar.heap = (uint64_t*)da;
            ar.tok = (uint32_t*)(ar.heap + 3 * long_total);
            ar.nxt = ar.tok + long_total;
            ar.prv = ar.nxt + long_total;
        }
    }
    ar.slot = slot;
    if (e == hipSuccess)
        hipLaunchKernelGGL(k_me_walk, dim3((uint32_t)gbpe_div_up(nchunks, ME_TPB)), dim3(ME_TPB), 0, s, d_in, n, t,
                           scratch, counts, base, nchunks, ar);
    hipLaunchKernelGGL(k_chunk_scan1, dim3((uint32_t)nblk), dim3(SCAN_TPB), 0, s, (const uint32_t*)counts, nchunks,
                       local, blocksum);
    hipLaunchKernelGGL(k_chunk_scan2, dim3(1), dim3(SCAN_TPB), 0, s, blocksum, nblk, total);
    hipLaunchKernelGGL(k_me_compact, dim3((uint32_t)gbpe_div_up(nchunks, 4)), dim3(256), 0, s, (const uint32_t*)scratch,
                       (const uint32_t*)counts, (const uint64_t*)base, (const uint32_t*)local,
                       (const uint64_t*)blocksum, nchunks, d_out, n);
    if (e == hipSuccess) e = hipGetLastError();
    uint64_t tot = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&tot, total, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess && tot <= out_cap && out && tot)
        e = hipMemcpy(out, d_out, tot * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    hipFree(da);
    hipFree(slot);
    if (e != hipSuccess) return gbpe_set_error(ctx, GBPE_E_DEVICE, "bpe encode failed: %s", hipGetErrorString(e));
    *n_out = tot;
    if (tot > out_cap) return gbpe_set_error(ctx, GBPE_E_CAPACITY, "bpe encode: output needs %llu tokens",
                                             (unsigned long long)tot);
    return GBPE_OK;
}
