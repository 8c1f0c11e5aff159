/*
 * bpe_oracle_inc.c — incremental CPU restatement of the reference training
 * loop.  TEST / FIXTURE INFRASTRUCTURE ONLY: it produces the full-length
 * merge lists that tests/golden/ pins the HIP path against (1 GiB corpora,
 * 32K-50K merges), which the full-recount restatement in bpe_oracle.c
 * (hours per 1 GiB run) cannot.  It is checked merge-for-merge and
 * symbol-for-symbol against bpe_oracle.c by tests/test_oracle_inc.py.
 * Never linked into, or called by, the product library.
 *
 * Semantics (toprakdeviren/gpu-bpe, src/bpe/train.wgsl), identical to
 * bpe_oracle.c:
 *   pair (i-1, i) counts iff !ws(i) and both tokens != 0     train.wgsl:393-399
 *   argmax: higher count, then smaller a<<16|b                train.wgsl:83-85, 204-318
 *   stop when count < 2 or the id would pass 0xFFFF           train.wgsl:345-348
 *   snapshot merge: hit(i) = !ws(i) & tok(i-1)==a & tok(i)==b;
 *     position i-1 of the ping buffer becomes new|ws in place,
 *     position i is dropped (a run of a==b collapses)         train.wgsl:475-500
 *   compaction bounded by the NEW count: the survivors whose old
 *     index is >= new_n are not written, so the last m slots keep
 *     the pong buffer's stale contents (the previous merge's input
 *     stream, after that merge's in-place A-side rewrite)     train.wgsl:605-607, 698, 727
 *
 * Data structures (not the GPU's): the stream is a doubly linked list of
 * nodes; per token, a lazily-compacted list of the nodes holding it; an exact
 * open-addressing pair-count table; a lazy max-heap of (count << 32 | ~pid).
 * A merge visits the occurrences of the rarer of its two tokens, the merge
 * sites' neighbourhoods, and the last ~5*count positions of the stream (the
 * stale-window bookkeeping).  Single threaded.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WSB 0x10000u
#define TMK 0xFFFFu
#define DEAD 0x80000000u
#define NIL 0xFFFFFFFFu

void oracle_heuristic_ws(const uint8_t* d, uint64_t n, uint32_t* out);   /* bpe_oracle.c */

static inline uint32_t fmix(uint32_t x) {
    x = (x ^ (x >> 16)) * 0x7feb352du;
    x = (x ^ (x >> 15)) * 0x846ca68bu;
    return x ^ (x >> 16);
}

/* ── exact pair counts ── */
typedef struct {
    uint32_t* key;
    uint32_t* cnt;
    uint32_t* mark;   /* epoch of the last change (one heap push per pid per merge) */
    uint64_t mask, used;
} ctab_t;

static int ct_init(ctab_t* t, int lg) {
    t->mask = (1ull << lg) - 1;
    t->used = 0;
    t->key = calloc(t->mask + 1, 4);
    t->cnt = calloc(t->mask + 1, 4);
    t->mark = calloc(t->mask + 1, 4);
    return t->key && t->cnt && t->mark ? 0 : -1;
}
static void ct_free(ctab_t* t) { free(t->key); free(t->cnt); free(t->mark); }
static uint64_t ct_slot(ctab_t* t, uint32_t k);
static int ct_grow(ctab_t* t) {
    ctab_t n;
    int lg = 0;
    while ((1ull << lg) < (t->mask + 1) * 2) ++lg;
    if (ct_init(&n, lg)) return -1;
    for (uint64_t i = 0; i <= t->mask; ++i)
        if (t->key[i]) {
            uint64_t s = ct_slot(&n, t->key[i]);
            n.key[s] = t->key[i];
            n.cnt[s] = t->cnt[i];
            n.mark[s] = t->mark[i];
            ++n.used;
        }
    ct_free(t);
    *t = n;
    return 0;
}
/* slot of k (existing or the empty slot where it would go) */
static uint64_t ct_slot(ctab_t* t, uint32_t k) {
    uint64_t i = fmix(k) & t->mask;
    while (t->key[i] && t->key[i] != k) i = (i + 1) & t->mask;
    return i;
}

/* ── lazy max-heap of (count << 32) | ~pid ── */
typedef struct { uint64_t* v; uint64_t n, cap; } heap_t;
static int hp_push(heap_t* h, uint64_t x) {
    if (h->n == h->cap) {
        uint64_t nc = h->cap ? 2 * h->cap : 1 << 20;
        uint64_t* nv = realloc(h->v, nc * 8);
        if (!nv) return -1;
        h->v = nv;
        h->cap = nc;
    }
    uint64_t i = h->n++;
    while (i) {
        uint64_t p = (i - 1) / 2;
        if (h->v[p] >= x) break;
        h->v[i] = h->v[p];
        i = p;
    }
    h->v[i] = x;
    return 0;
}
static uint64_t hp_pop(heap_t* h) {
    uint64_t top = h->v[0], x = h->v[--h->n], i = 0;
    for (;;) {
        uint64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && h->v[c + 1] > h->v[c]) ++c;
        if (h->v[c] <= x) break;
        h->v[i] = h->v[c];
        i = c;
    }
    if (h->n) h->v[i] = x;
    return top;
}

/* ── per-token occurrence lists ── */
typedef struct { uint32_t* v; uint32_t n, cap; } occ_t;
static int oc_push(occ_t* o, uint32_t x) {
    if (o->n == o->cap) {
        uint32_t nc = o->cap ? (o->cap < (1u << 30) ? 2 * o->cap : o->cap + (1u << 28)) : 16;
        uint32_t* nv = realloc(o->v, (uint64_t)nc * 4);
        if (!nv) return -1;
        o->v = nv;
        o->cap = nc;
    }
    o->v[o->n++] = x;
    return 0;
}

typedef struct {
    uint32_t *tok, *prv, *nxt;
    uint8_t* fl;          /* bit0 site, bit1 in E, bit2 seen in this occurrence scan */
    uint32_t head, tail;
    uint64_t n;           /* live nodes */
    uint32_t* freel;      /* recycled node ids */
    uint64_t nfree, cap;
    occ_t occ[65536];
    uint64_t tokcnt[65536];
    ctab_t ct;
    heap_t hp;
    uint32_t epoch;
    uint32_t* chg;        /* pids changed in this merge */
    uint64_t nchg, chg_cap;
    int err;
} st_t;

static void note_change(st_t* S, uint64_t slot) {
    if (S->ct.mark[slot] == S->epoch) return;
    S->ct.mark[slot] = S->epoch;
    if (S->nchg == S->chg_cap) {
        uint64_t nc = S->chg_cap ? 2 * S->chg_cap : 1 << 16;
        uint32_t* nv = realloc(S->chg, nc * 4);
        if (!nv) { S->err = -2; return; }
        S->chg = nv;
        S->chg_cap = nc;
    }
    S->chg[S->nchg++] = S->ct.key[slot];
}

static void pair_add(st_t* S, uint32_t pid, int d) {
    uint64_t s = ct_slot(&S->ct, pid);
    if (!S->ct.key[s]) {
        if (d < 0) { S->err = -7; return; }   /* removing a pair that was never counted */
        S->ct.key[s] = pid;
        S->ct.cnt[s] = 0;
        S->ct.mark[s] = 0;
        if (++S->ct.used * 2 > S->ct.mask) {
            if (ct_grow(&S->ct)) { S->err = -2; return; }
            s = ct_slot(&S->ct, pid);
        }
    }
    if (d < 0 && S->ct.cnt[s] == 0) { S->err = -7; return; }
    S->ct.cnt[s] += (uint32_t)d;
    note_change(S, s);
}

/* the pair ending at node e (the symbol before it in the stream, and e) */
static inline uint32_t pair_at(const st_t* S, uint32_t e) {
    uint32_t x = S->tok[e];
    if (x & WSB) return 0;
    uint32_t p = S->prv[e];
    if (p == NIL) return 0;
    uint32_t tp = S->tok[p] & TMK, te = x & TMK;
    return (tp && te) ? (tp << 16) | te : 0;
}

static uint32_t node_alloc(st_t* S) {
    if (S->nfree) return S->freel[--S->nfree];
    S->err = -7;   /* the stream never outgrows its initial length */
    return NIL;
}
static void node_free(st_t* S, uint32_t j) {
    S->tok[j] = DEAD;
    S->freel[S->nfree++] = j;
}
static void unlink_node(st_t* S, uint32_t j) {
    uint32_t p = S->prv[j], q = S->nxt[j];
    if (p != NIL) S->nxt[p] = q; else S->head = q;
    if (q != NIL) S->prv[q] = p; else S->tail = p;
}

int oracle_train_inc(const uint8_t* bytes, uint64_t n, const uint8_t* ws_ext, uint32_t target, uint32_t vocab_size,
                     uint32_t next_id, int exact, uint32_t max_merges, uint32_t* merges_out, uint32_t* n_merges,
                     uint32_t* early_stop, uint32_t* final_syms, uint64_t* final_n, uint64_t* tail_total) {
    if (n == 0) return -6;
    if (n >= 0xFFFFFFF0ull) return -1;
    st_t* S = calloc(1, sizeof(st_t));
    if (!S) return -2;
    int rc = 0;
    uint32_t *save = NULL, *nsave = NULL, *tailnodes = NULL, *sites = NULL, *E = NULL;
    uint64_t save_cap = 0, sites_cap = 0, E_cap = 0;
    S->cap = n;
    S->tok = malloc(n * 4);
    S->prv = malloc(n * 4);
    S->nxt = malloc(n * 4);
    S->fl = calloc(n, 1);
    S->freel = malloc(n * 4);
    if (!S->tok || !S->prv || !S->nxt || !S->fl || !S->freel || ct_init(&S->ct, 20)) { rc = -2; goto out; }
    if (ws_ext) {
        for (uint64_t i = 0; i < n; ++i) S->tok[i] = bytes[i] | (ws_ext[i] ? WSB : 0u);
    } else {
        oracle_heuristic_ws(bytes, n, S->tok);
    }
    for (uint64_t i = 0; i < n; ++i) {
        S->prv[i] = i ? (uint32_t)(i - 1) : NIL;
        S->nxt[i] = i + 1 < n ? (uint32_t)(i + 1) : NIL;
        S->tokcnt[S->tok[i] & TMK]++;
    }
    for (uint32_t t = 1; t < 256; ++t)
        if (S->tokcnt[t]) {
            S->occ[t].v = malloc(S->tokcnt[t] * 4);
            if (!S->occ[t].v) { rc = -2; goto out; }
            S->occ[t].cap = (uint32_t)S->tokcnt[t];
        }
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t t = S->tok[i] & TMK;
        if (t) S->occ[t].v[S->occ[t].n++] = (uint32_t)i;
    }
    S->head = 0;
    S->tail = (uint32_t)(n - 1);
    S->n = n;
    S->epoch = 1;
    for (uint64_t i = 1; i < n; ++i) {
        uint32_t pid = pair_at(S, (uint32_t)i);
        if (pid) pair_add(S, pid, 1);
    }
    for (uint64_t i = 0; i < S->nchg; ++i) {
        uint64_t s = ct_slot(&S->ct, S->chg[i]);
        if (hp_push(&S->hp, ((uint64_t)S->ct.cnt[s] << 32) | (uint32_t)~S->chg[i])) { rc = -2; goto out; }
    }
    S->nchg = 0;
    if (S->err) { rc = S->err; goto out; }

    uint32_t needed = target > vocab_size ? target - vocab_size : 0;
    if (max_merges && max_merges < needed) needed = max_merges;
    uint32_t nxt = next_id, done = 0, stop = 0;
    uint64_t tail_sum = 0;
    /* stale source of the coming merge: the previous merge's input stream, last
     * save_len positions starting at save_base; before the first merge the pong
     * buffer is all zeros (WebGPU zero-initialised) */
    int save_zero = 1;
    uint64_t save_base = 0, save_len = 0;
    while (done < needed) {
        /* ── selection ── */
        uint32_t mc = 0, pid = 0;
        while (S->hp.n) {
            uint64_t top = S->hp.v[0];
            uint32_t c = (uint32_t)(top >> 32), k = ~(uint32_t)top;
            uint64_t s = ct_slot(&S->ct, k);
            if (S->ct.key[s] == k && S->ct.cnt[s] == c && c > 0) { mc = c; pid = k; break; }
            hp_pop(&S->hp);   /* stale entry */
        }
        if (mc < 2 || nxt > TMK) { stop = 1; break; }
        const uint32_t a = pid >> 16, b = pid & TMK, nw = nxt;
        ++S->epoch;
        /* ── merge sites: the occurrences of the rarer token ── */
        const int scan_b = S->tokcnt[b] <= S->tokcnt[a];
        const uint32_t T = scan_b ? b : a;
        occ_t* L = &S->occ[T];
        uint64_t ns = 0;
        if (sites_cap < mc) {
            free(sites);
            sites_cap = (uint64_t)mc * 2;
            sites = malloc(sites_cap * 4);
            if (!sites) { rc = -2; goto out; }
        }
        uint32_t w = 0;
        for (uint32_t q = 0; q < L->n; ++q) {
            uint32_t x = L->v[q];
            if ((S->tok[x] & (TMK | DEAD)) != T || (S->fl[x] & 4)) continue;   /* stale or duplicate entry */
            S->fl[x] |= 4;
            L->v[w++] = x;
            uint32_t j = NIL;
            if (scan_b) {
                if (!(S->tok[x] & WSB) && S->prv[x] != NIL && (S->tok[S->prv[x]] & TMK) == a) j = x;
            } else {
                uint32_t y = S->nxt[x];
                if (y != NIL && !(S->tok[y] & WSB) && (S->tok[y] & (TMK | DEAD)) == b) j = y;
            }
            if (j != NIL && !(S->fl[j] & 1)) {
                if (ns == mc) { rc = -7; goto out; }   /* more sites than the counted pairs */
                S->fl[j] |= 1;
                sites[ns++] = j;
            }
        }
        L->n = w;
        for (uint32_t q = 0; q < w; ++q) S->fl[L->v[q]] &= (uint8_t)~4;
        if (ns != mc) { rc = -7; goto out; }
        /* ── old pairs around every site (snapshot) ── */
        uint64_t nE = 0;
        if (E_cap < 3 * ns) {
            free(E);
            E_cap = 3 * ns * 2;
            E = malloc(E_cap * 4);
            if (!E) { rc = -2; goto out; }
        }
        for (uint64_t i = 0; i < ns; ++i) {
            uint32_t j = sites[i], c3[3] = {S->prv[j], j, S->nxt[j]};
            for (int k = 0; k < 3; ++k)
                if (c3[k] != NIL && !(S->fl[c3[k]] & 2)) {
                    S->fl[c3[k]] |= 2;
                    E[nE++] = c3[k];
                }
        }
        for (uint64_t i = 0; i < nE; ++i) {
            uint32_t p = pair_at(S, E[i]);
            if (p) pair_add(S, p, -1);
        }
        /* ── the last positions of the input stream (stale-window bookkeeping) ── */
        const uint64_t nold = S->n, new_n = nold - mc;
        uint64_t Lt = 0;
        if (!exact) {
            Lt = 5ull * mc + 8;
            if (Lt > nold) Lt = nold;
            if (save_cap < 2 * Lt) {
                free(tailnodes);
                free(nsave);
                save_cap = 4 * Lt;
                tailnodes = malloc(save_cap * 4);
                nsave = malloc(save_cap * 4);
                if (!tailnodes || !nsave) { rc = -2; goto out; }
                if (!save_zero) {   /* keep the current save: copy into a grown buffer */
                    uint32_t* ns2 = malloc(save_cap * 4);
                    if (!ns2) { rc = -2; goto out; }
                    memcpy(ns2, save, save_len * 4);
                    free(save);
                    save = ns2;
                } else {
                    free(save);
                    save = malloc(save_cap * 4);
                    if (!save) { rc = -2; goto out; }
                }
            }
            uint32_t x = S->tail;
            for (uint64_t k = Lt; k-- > 0;) {
                tailnodes[k] = x;
                x = S->prv[x];
            }
        }
        /* ── token counts and occurrence lists; in-place A-side rewrite ── */
        for (uint64_t i = 0; i < ns; ++i) S->tokcnt[b]--;
        for (uint64_t i = 0; i < ns; ++i) {
            uint32_t p = S->prv[sites[i]];
            if (!(S->fl[p] & 1)) {
                S->tokcnt[a]--;
                S->tokcnt[nw]++;
                if (oc_push(&S->occ[nw], p)) { rc = -2; goto out; }
            }
        }
        for (uint64_t i = 0; i < ns; ++i) {
            uint32_t p = S->prv[sites[i]];
            S->tok[p] = nw | (S->tok[p] & WSB);
        }
        if (!exact)   /* the ping buffer after the merge: the next merge's stale source */
            for (uint64_t k = 0; k < Lt; ++k) nsave[k] = S->tok[tailnodes[k]];
        /* ── drop the B-sides; new pairs around every site ── */
        for (uint64_t i = 0; i < ns; ++i) unlink_node(S, sites[i]);
        S->n = new_n;
        for (uint64_t i = 0; i < nE; ++i) {
            uint32_t e = E[i];
            if (S->fl[e] & 1) continue;
            uint32_t p = pair_at(S, e);
            if (p) pair_add(S, p, 1);
        }
        for (uint64_t i = 0; i < nE; ++i) S->fl[E[i]] &= (uint8_t)~2;
        /* ── the reference compaction: survivors with old index >= new_n are not
         *    written; the stale window takes their place ── */
        uint64_t m = 0;
        if (!exact) {
            /* survivors among old positions [new_n, nold) = tailnodes[Lt - mc, Lt) */
            uint32_t first_drop = NIL;
            for (uint64_t k = Lt - mc; k < Lt; ++k) {
                uint32_t d = tailnodes[k];
                if (S->fl[d] & 1) continue;
                if (first_drop == NIL) first_drop = d;
                ++m;
                uint32_t p = pair_at(S, d);
                if (p) pair_add(S, p, -1);
            }
            if (m) {
                /* they are the last m nodes of the list */
                uint32_t keep_tail = S->prv[first_drop];
                uint64_t cnt = 0;
                for (uint32_t d = first_drop; d != NIL;) {
                    uint32_t nx = S->nxt[d];
                    S->tokcnt[S->tok[d] & TMK]--;
                    node_free(S, d);
                    d = nx;
                    ++cnt;
                }
                if (cnt != m) { rc = -7; goto out; }
                S->tail = keep_tail;
                if (keep_tail != NIL) S->nxt[keep_tail] = NIL; else S->head = NIL;
                /* window: stale positions [new_n - m, new_n) */
                for (uint64_t k = 0; k < m; ++k) {
                    const uint64_t pos = new_n - m + k;
                    uint32_t v = 0;
                    if (!save_zero) {
                        if (pos < save_base || pos - save_base >= save_len) { rc = -7; goto out; }
                        v = save[pos - save_base];
                    }
                    uint32_t wn = node_alloc(S);
                    if (wn == NIL) { rc = -7; goto out; }
                    S->tok[wn] = v;
                    S->prv[wn] = S->tail;
                    S->nxt[wn] = NIL;
                    if (S->tail != NIL) S->nxt[S->tail] = wn; else S->head = wn;
                    S->tail = wn;
                    S->tokcnt[v & TMK]++;
                    if ((v & TMK) && oc_push(&S->occ[v & TMK], wn)) { rc = -2; goto out; }
                    uint32_t p = pair_at(S, wn);
                    if (p) pair_add(S, p, 1);
                }
            }
            /* this merge's input (after its in-place rewrite) is the next stale source */
            uint32_t* t2 = save;
            save = nsave;
            nsave = t2;
            save_base = nold - Lt;
            save_len = Lt;
            save_zero = 0;
        }
        for (uint64_t i = 0; i < ns; ++i) {
            S->fl[sites[i]] &= (uint8_t)~1;
            node_free(S, sites[i]);
        }
        tail_sum += m;
        if (S->err) { rc = S->err; goto out; }
        /* ── heap: one push per changed pid ── */
        for (uint64_t i = 0; i < S->nchg; ++i) {
            uint64_t s = ct_slot(&S->ct, S->chg[i]);
            if (S->ct.cnt[s] && hp_push(&S->hp, ((uint64_t)S->ct.cnt[s] << 32) | (uint32_t)~S->chg[i])) { rc = -2; goto out; }
        }
        S->nchg = 0;
        if (S->hp.n > 4 * S->ct.used + (1u << 22)) {   /* drop stale entries: rebuild from the table */
            S->hp.n = 0;
            for (uint64_t s = 0; s <= S->ct.mask; ++s)
                if (S->ct.key[s] && S->ct.cnt[s] && hp_push(&S->hp, ((uint64_t)S->ct.cnt[s] << 32) | (uint32_t)~S->ct.key[s])) {
                    rc = -2;
                    goto out;
                }
        }
        merges_out[4 * done + 0] = a;
        merges_out[4 * done + 1] = b;
        merges_out[4 * done + 2] = nw;
        merges_out[4 * done + 3] = mc;
        ++done;
        ++nxt;
    }
    *n_merges = done;
    if (early_stop) *early_stop = stop;
    if (final_n) *final_n = S->n;
    if (tail_total) *tail_total = tail_sum;
    if (final_syms) {
        uint64_t k = 0;
        for (uint32_t x = S->head; x != NIL; x = S->nxt[x]) final_syms[k++] = S->tok[x];
        if (k != S->n) rc = -7;
    }
out:
    free(save); free(nsave); free(tailnodes); free(sites); free(E);
    for (int t = 0; t < 65536; ++t) free(S->occ[t].v);
    free(S->tok); free(S->prv); free(S->nxt); free(S->fl); free(S->freel); free(S->chg); free(S->hp.v);
    ct_free(&S->ct);
    free(S);
    return rc;
}

/* GPT-4 rule word starts (pre_tokenizer.mjs:226-292, byte mapping :497-506)
 * for ASCII-only input, with the 128 codepoint classes supplied by the caller
 * (oracle/bpe_oracle.py pt_classify).  Returns -1 on a non-ASCII byte. */
enum { PL = 0, PD = 1, PW = 2, PP = 3, PS = 4, PN = 5, PO = 6 };
int oracle_gpt4_ws_ascii(const uint8_t* b, uint64_t n, const uint8_t* cls, uint8_t* out) {
    for (uint64_t i = 0; i < n; ++i)
        if (b[i] >= 0x80) return -1;
    memset(out, 0, n);
    if (!n) return 0;
    out[0] = 1;
    uint64_t i = 1, run = 1;   /* run: length of the digit run ending at i-1 */
    run = cls[b[0]] == PD ? 1 : 0;
#define PSY(c) ((c) == PP || (c) == PS)
    while (i < n) {
        const uint8_t pc = cls[b[i - 1]], cc = cls[b[i]];
        if (cc == PN || pc == PN) { out[i] = 1; goto next; }
        if (cc == PW) { if (pc != PW) out[i] = 1; goto next; }
        if (pc == PW) goto next;
        if (pc == PL && b[i] == 0x27) {   /* matchContraction (:85-114) */
            uint64_t k = 0;
            if (i + 1 < n) {
                uint8_t nx = b[i + 1];
                int after1 = i + 2 >= n || cls[b[i + 2]] != PL;
                if ((nx == 's' || nx == 'S' || nx == 't' || nx == 'T' || nx == 'm' || nx == 'M' || nx == 'd' ||
                     nx == 'D') && after1)
                    k = 2;
                else if (i + 2 < n) {
                    uint8_t nn = b[i + 2];
                    int after2 = i + 3 >= n || cls[b[i + 3]] != PL;
                    if (after2 && (((nx == 'r' || nx == 'R') && (nn == 'e' || nn == 'E')) ||
                                   ((nx == 'v' || nx == 'V') && (nn == 'e' || nn == 'E')) ||
                                   ((nx == 'l' || nx == 'L') && (nn == 'l' || nn == 'L'))))
                        k = 3;
                }
            }
            if (k) {
                i += k;
                run = cls[b[i - 1]] == PD ? 1 : 0;   /* contraction letters: never digits */
                continue;
            }
        }
        if ((pc == PL && cc == PD) || (pc == PD && cc == PL) || (pc == PL && PSY(cc)) || (PSY(pc) && cc == PL) ||
            (PSY(pc) && cc == PD) || (pc == PD && PSY(cc))) {
            out[i] = 1;
            goto next;
        }
        if (cc == PD && pc == PD) {
            if (run % 3 == 0) out[i] = 1;
        }
    next:
        run = cls[b[i]] == PD ? (cls[b[i - 1]] == PD ? run + 1 : 1) : 0;
        ++i;
    }
#undef PSY
    return 0;
}
