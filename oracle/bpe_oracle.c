/*
 * bpe_oracle.c — C restatement of the reference algorithm.  TEST / BENCH
 * INFRASTRUCTURE ONLY: used by tests/ as the large-input checker and by
 * bench.py as the `cpu_baseline` leg ("kind": "port").  Never linked into,
 * or called by, the product library.
 *
 * It restates, per merge, exactly what the reference does on the GPU
 * (toprakdeviren/gpu-bpe, src/bpe/train.wgsl + training-pipeline.js:178-222):
 *   full pair recount of the whole stream   (bpe_clear_table + bpe_pair_count_b, train.wgsl:188-202, 366-431)
 *   deterministic argmax                    (bpe_find_max_pair4 + _final_det, train.wgsl:83-85, 204-318)
 *   stop on count < 2 or id > 0xFFFF        (bpe_setup_merge, train.wgsl:340-364)
 *   snapshot merge + in-place A-side write  (bpe_merge_reduce_b, train.wgsl:457-520)
 *   compaction bounded by the NEW count     (scan + bpe_finalize_compact_b, train.wgsl:605-607, 686-730)
 * with exact counting (no hash-probe drops).  OpenMP over stream ranges.
 *
 * The chunked greedy trie walk restates tokenize.wgsl:88-175 over the
 * reference's {firstChild,numChildren,tokenId} nodes and sorted edges with
 * the same branchless lower-bound child search (tokenize.wgsl:69-86).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define WS 0x10000u
#define TM 0xFFFFu
#define INVALID 0xFFFFFFFFu

static inline uint32_t fmix(uint32_t x) {
    x = (x ^ (x >> 16)) * 0x7feb352du;
    x = (x ^ (x >> 15)) * 0x846ca68bu;
    return x ^ (x >> 16);
}

/* open-addressing exact counter: key 0 = empty (pid 0 never counted) */
typedef struct { uint32_t* key; uint32_t* val; uint32_t mask; uint32_t used; } tab_t;

static void tab_init(tab_t* t, uint32_t log2) {
    t->mask = (1u << log2) - 1;
    t->key = (uint32_t*)calloc((size_t)t->mask + 1, 4);
    t->val = (uint32_t*)calloc((size_t)t->mask + 1, 4);
    t->used = 0;
}
static void tab_free(tab_t* t) { free(t->key); free(t->val); }
static void tab_clear(tab_t* t) {
    memset(t->key, 0, ((size_t)t->mask + 1) * 4);
    memset(t->val, 0, ((size_t)t->mask + 1) * 4);
    t->used = 0;
}
static void tab_add(tab_t* t, uint32_t k, uint32_t v);
static void tab_grow(tab_t* t) {
    tab_t n;
    uint32_t lg = 0;
    while ((1u << lg) < (t->mask + 1) * 2) ++lg;
    tab_init(&n, lg);
    for (uint32_t i = 0; i <= t->mask; ++i)
        if (t->key[i]) tab_add(&n, t->key[i], t->val[i]);
    tab_free(t);
    *t = n;
}
static void tab_add(tab_t* t, uint32_t k, uint32_t v) {
    uint32_t i = fmix(k) & t->mask;
    for (;;) {
        if (t->key[i] == k) { t->val[i] += v; return; }
        if (t->key[i] == 0) {
            t->key[i] = k; t->val[i] = v;
            if (++t->used * 2 > t->mask) tab_grow(t);
            return;
        }
        i = (i + 1) & t->mask;
    }
}

/* full recount + argmax; returns best count, *best_pid.
 * local[t*T + p]: thread t's counts for hash partition p; thread p then sums
 * partition p over all threads (work = entries, not T x table size). */
static uint32_t count_and_select(const uint32_t* s, uint64_t n, int T, tab_t* local, tab_t* part, uint32_t* best_pid) {
    uint32_t bc_all = 0, bp_all = 0;
#pragma omp parallel num_threads(T)
    {
        int t = omp_get_thread_num();
        for (int p = 0; p < T; ++p) tab_clear(&local[t * T + p]);
        uint64_t lo = 1 + (n > 1 ? (n - 1) * (uint64_t)t / T : 0), hi = 1 + (n > 1 ? (n - 1) * (uint64_t)(t + 1) / T : 0);
        for (uint64_t i = lo; i < hi; ++i) {
            uint32_t x1 = s[i];
            if (x1 & WS) continue;
            uint32_t a = s[i - 1] & TM, b = x1 & TM;
            if (a && b) {
                uint32_t k = (a << 16) | b;
                tab_add(&local[t * T + (fmix(k) >> 24) % (uint32_t)T], k, 1);
            }
        }
#pragma omp barrier
        tab_clear(&part[t]);
        for (int u = 0; u < T; ++u) {
            tab_t* L = &local[u * T + t];
            for (uint32_t i = 0; i <= L->mask; ++i)
                if (L->key[i]) tab_add(&part[t], L->key[i], L->val[i]);
        }
        uint32_t bc = 0, bp = 0;
        tab_t* P = &part[t];
        for (uint32_t i = 0; i <= P->mask; ++i) {
            uint32_t k = P->key[i], c = P->val[i];
            if (k && (c > bc || (c == bc && k < bp))) { bc = c; bp = k; }
        }
#pragma omp critical
        {
            if (bc > bc_all || (bc == bc_all && bc && bp < bp_all)) { bc_all = bc; bp_all = bp; }
        }
    }
    *best_pid = bp_all;
    return bc_all;
}

/* one merge cur -> oth; returns new count.  hit[i] = pair (i-1,i) == (a,b) */
static uint64_t merge_step(uint32_t* cur, uint32_t* oth, uint64_t n, uint32_t a, uint32_t b, uint32_t nw, int exact,
                           int T, uint8_t* hit, uint64_t* part_cnt, uint64_t* tail) {
#pragma omp parallel num_threads(T)
    {
        int t = omp_get_thread_num();
        uint64_t lo = n * (uint64_t)t / T, hi = n * (uint64_t)(t + 1) / T;
        uint64_t c = 0;
        for (uint64_t i = lo; i < hi; ++i) {
            uint8_t h = 0;
            if (i >= 1) {
                uint32_t x1 = cur[i];
                h = !(x1 & WS) && (cur[i - 1] & TM) == a && (x1 & TM) == b;
            }
            hit[i] = h;
            c += !h;
        }
        part_cnt[t] = c;
    }
    uint64_t total = 0;
    for (int t = 0; t < T; ++t) { uint64_t c = part_cnt[t]; part_cnt[t] = total; total += c; }
    const uint64_t new_n = total;
    const uint64_t lim = exact ? n : new_n;
    uint64_t dropped = 0;
#pragma omp parallel num_threads(T) reduction(+ : dropped)
    {
        int t = omp_get_thread_num();
        uint64_t lo = n * (uint64_t)t / T, hi = n * (uint64_t)(t + 1) / T;
        uint64_t d = part_cnt[t];
        for (uint64_t i = lo; i < hi; ++i) {
            uint32_t x = cur[i];
            if (i + 1 < n && hit[i + 1]) x = nw | (x & WS);   /* A-side rewrite (snapshot: hit[] computed first) */
            if (!hit[i]) {
                if (i < lim) oth[d] = x; else ++dropped;
                ++d;
            }
        }
    }
    /* in-place rewrite of the ping buffer after every read */
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t i = 0; i < (int64_t)n - 1; ++i)
        if (hit[i + 1]) cur[i] = nw | (cur[i] & WS);
    *tail += dropped;
    return new_n;
}

void oracle_heuristic_ws(const uint8_t* d, uint64_t n, uint32_t* out) {
#define CLS(t) ((t) == 0x0Au ? 4u : (t) == 0x20u ? 2u : ((t) - 0x30u <= 9u) ? 1u : (t) >= 0x80u ? 0u : (((t) | 0x20u) - 0x61u <= 25u) ? 0u : 3u)
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint32_t tk = d[i], ws;
        if (i == 0) ws = 1;
        else {
            uint32_t c = CLS(tk), p = CLS((uint32_t)d[i - 1]);
            ws = c != p;
            if (p == 2u && (c == 0u || c == 1u)) ws = 0;
            if (c == 2u && p != 2u) ws = 1;
            if (p == 4u || c == 4u) ws = 1;
        }
        out[i] = tk | (ws ? WS : 0u);
    }
#undef CLS
}

/* returns number of merges; merges_out = [a,b,id,count] x n.  final stream optional. */
int oracle_train(const uint8_t* bytes, uint64_t n, const uint8_t* ws_ext, uint32_t target, uint32_t vocab_size,
                 uint32_t next_id, int exact, uint32_t max_merges, int threads, uint32_t* merges_out,
                 uint32_t* n_merges, uint32_t* early_stop, uint32_t* final_syms, uint64_t* final_n,
                 uint64_t* tail_total) {
    if (n == 0) return -6;
    int T = threads > 0 ? threads : omp_get_max_threads();
    uint32_t* A = (uint32_t*)malloc(n * 4);
    uint32_t* B = (uint32_t*)calloc(n, 4);          /* WebGPU zero-initialised pong buffer */
    uint8_t* hit = (uint8_t*)malloc(n + 1);
    uint64_t* part = (uint64_t*)calloc((size_t)T + 1, 8);
    tab_t* local = (tab_t*)calloc((size_t)T * T, sizeof(tab_t));
    tab_t* parts = (tab_t*)calloc((size_t)T, sizeof(tab_t));
    for (int t = 0; t < T * T; ++t) tab_init(&local[t], 10);
    for (int t = 0; t < T; ++t) tab_init(&parts[t], 12);
    if (ws_ext) {
        for (uint64_t i = 0; i < n; ++i) A[i] = bytes[i] | (ws_ext[i] ? WS : 0u);
    } else {
        oracle_heuristic_ws(bytes, n, A);
    }
    uint32_t needed = target > vocab_size ? target - vocab_size : 0;
    if (max_merges && max_merges < needed) needed = max_merges;
    uint32_t *cur = A, *oth = B, nxt = next_id, done = 0, stop = 0;
    uint64_t len = n, tail = 0;
    while (done < needed) {
        uint32_t pid = 0;
        uint32_t mc = count_and_select(cur, len, T, local, parts, &pid);
        if (mc < 2 || nxt > TM) { stop = 1; break; }
        uint32_t a = pid >> 16, b = pid & TM;
        len = merge_step(cur, oth, len, a, b, nxt, exact, T, hit, part, &tail);
        merges_out[4 * done + 0] = a;
        merges_out[4 * done + 1] = b;
        merges_out[4 * done + 2] = nxt;
        merges_out[4 * done + 3] = mc;
        ++done; ++nxt;
        uint32_t* tmp = cur; cur = oth; oth = tmp;
    }
    *n_merges = done;
    if (early_stop) *early_stop = stop;
    if (final_n) *final_n = len;
    if (final_syms) memcpy(final_syms, cur, len * 4);
    if (tail_total) *tail_total = tail;
    for (int t = 0; t < T * T; ++t) tab_free(&local[t]);
    for (int t = 0; t < T; ++t) tab_free(&parts[t]);
    free(local); free(parts); free(part); free(hit); free(A); free(B);
    return 0;
}

/* ── chunked greedy trie walk ─────────────────────────────────────────── */
static inline uint32_t find_child(const uint32_t* edges, uint32_t first, uint32_t num, uint32_t sym) {
    uint32_t lo = 0, m = num;
    while (m > 0) {
        uint32_t half = m >> 1, mid = lo + half;
        int less = (edges[(first + mid) * 2] & 0xFFu) < sym;
        lo = less ? mid + 1 : lo;
        m = less ? m - half - 1 : half;
    }
    if (lo < num && (edges[(first + lo) * 2] & 0xFFu) == sym) return edges[(first + lo) * 2 + 1];
    return INVALID;
}

static uint64_t walk_chunk(const uint8_t* d, uint64_t c0, uint64_t ce, const uint32_t* nodes, const uint32_t* edges,
                           const uint32_t* lut, uint32_t* out) {
    uint64_t pos = c0, cnt = 0;
    while (pos < ce) {
        uint32_t cn = 0, lmt = INVALID, depth = 0;
        uint64_t lmp = pos, wp = pos;
        while (wp < ce) {
            uint32_t bv = d[wp], nn;
            if (depth == 0) nn = lut[bv];
            else nn = find_child(edges, nodes[cn * 3], nodes[cn * 3 + 1] & 0xFFFFu, bv);
            if (nn == INVALID) break;
            cn = nn; ++wp; ++depth;
            uint32_t ti = nodes[cn * 3 + 2];
            if (ti != INVALID) { lmt = ti; lmp = wp; }
        }
        if (lmt != INVALID) { if (out) out[cnt] = lmt; ++cnt; pos = lmp; }
        else { if (out) out[cnt] = d[pos]; ++cnt; ++pos; }
    }
    return cnt;
}

/* two passes over chunks (count, then write); out may be NULL to only count */
uint64_t oracle_encode(const uint8_t* d, uint64_t n, const uint32_t* nodes, uint32_t n_nodes, const uint32_t* edges,
                       uint32_t chunk, int threads, uint32_t* out) {
    (void)n_nodes;
    if (n == 0) return 0;
    int T = threads > 0 ? threads : omp_get_max_threads();
    uint32_t lut[256];
    for (int c = 0; c < 256; ++c) lut[c] = INVALID;
    uint32_t rfc = nodes[0], rnc = nodes[1] & 0xFFFFu;
    for (uint32_t k = 0; k < rnc && k < 256; ++k) lut[edges[(rfc + k) * 2] & 0xFFu] = edges[(rfc + k) * 2 + 1];
    uint64_t nch = (n + chunk - 1) / chunk;
    uint64_t* cnt = (uint64_t*)malloc((nch + 1) * 8);
#pragma omp parallel for num_threads(T) schedule(dynamic, 64)
    for (int64_t c = 0; c < (int64_t)nch; ++c) {
        uint64_t c0 = (uint64_t)c * chunk, ce = c0 + chunk < n ? c0 + chunk : n;
        cnt[c] = walk_chunk(d, c0, ce, nodes, edges, lut, NULL);
    }
    uint64_t total = 0;
    for (uint64_t c = 0; c < nch; ++c) { uint64_t v = cnt[c]; cnt[c] = total; total += v; }
    if (out) {
#pragma omp parallel for num_threads(T) schedule(dynamic, 64)
        for (int64_t c = 0; c < (int64_t)nch; ++c) {
            uint64_t c0 = (uint64_t)c * chunk, ce = c0 + chunk < n ? c0 + chunk : n;
            walk_chunk(d, c0, ce, nodes, edges, lut, out + cnt[c]);
        }
    }
    free(cnt);
    return total;
}

int oracle_max_threads(void) { return omp_get_max_threads(); }
