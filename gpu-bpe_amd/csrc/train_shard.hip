// Sharded training (gbpe_shard_*, gbpe_comm_*, gbpe_shard_step_comm): one rank per
// GPU, a replica of the global pair table per rank, one exchange record per merge.
// Host loop: gpu-bpe_amd/gpubpe/sharded.py.  Shares the trainer (trainer.h) with train.hip.

#include "trainer.h"

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
    const uint32_t zn = zone ? (uint32_t)t->n - t->h_st->B : 0u;   // the zone only shrinks within a step
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
