"""numpy model of one rank of the sharded trainer — TEST INFRASTRUCTURE ONLY.

Implements the backend interface of ``gpubpe.sharded.ShardedTrainer`` with
plain numpy, record for record what csrc/train_shard.hip's gbpe_shard_* kernels
write, so the orchestration and the exchange protocol (window cut, owner
rank, offsets, stall/undo) are tested over gloo on CPU against the
single-stream oracle (oracle/bpe_oracle.py, the reference semantics).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-bpe_amd"))

import bpe_oracle as O  # noqa: E402
from gpubpe.sharded import (HDR, H_A, H_ACTIVE, H_B, H_HASLAST, H_ID, H_KEPT, H_L, H_LASTSYM, H_LN,  # noqa: E402
                            H_M, H_MC, H_SURV, H_W)

WS, TM = O.WORD_START_BIT, O.TOKEN_MASK


def _pairs(s: np.ndarray) -> dict:
    u, c = O.count_pairs(s)
    return dict(zip(u.tolist(), c.tolist()))


class ModelShardBackend:
    def __init__(self, data: bytes, word_starts, rank: int, world: int, target_vocab: int, exact: bool = False):
        self.rank, self.world = rank, world
        self.exact = exact
        sym = O.prepare_symbols(data, word_starts)
        self.ln = sym.shape[0]
        self.cap = 0
        self.sym0 = sym
        self.counts: dict = {}
        self.next_id = 256
        self.needed = target_vocab - 256
        self.done_total = 0
        self.stop = False
        self.events = {"window_multi_rank": 0, "owner_not_last": 0, "empty_ranks": 0}

    # ── setup ──
    def local_len(self):
        return self.ln

    def set_layout(self, lens):
        self.lens = list(lens)
        self.gn = sum(lens)
        self.off = sum(lens[: self.rank])
        self.poff, self.pln = self.off, self.ln
        self.cap = self.ln + self.gn + 16
        self.cur = np.zeros(self.cap, np.uint32)
        self.oth = np.zeros(self.cap, np.uint32)          # zero-initialised like the reference's buffers
        self.cur[: self.ln] = self.sym0

    def export_counts(self, device):
        import torch
        p = _pairs(self.cur[: self.ln])
        arr = np.array(sorted(p.items()), dtype=np.int64).reshape(-1, 2).astype(np.uint32).view(np.int32)
        return torch.from_numpy(arr.copy())

    def import_counts(self, allp, counts, pmax):
        a = allp.cpu().numpy().view(np.uint32).reshape(self.world, pmax, 2)
        self.counts = {}
        for r in range(self.world):
            for pid, c in a[r, : counts[r]].tolist():
                self.counts[pid] = self.counts.get(pid, 0) + c

    # ── one step ──
    def step_begin(self, max_merges):
        self.budget = max_merges
        self.log = []
        self.stalled = False
        self.need = (0, 0)
        self.peak = (0, 0)
        self.active = False

    def _select(self):
        best = None
        for pid, c in self.counts.items():
            if c <= 0:
                continue
            if best is None or c > best[0] or (c == best[0] and pid < best[1]):
                best = (c, pid)
        return best if best else (0, 0)

    def phase1(self, k, send, C, Cw):
        rec = np.zeros(send.numel(), np.uint32)
        self.active = False
        if not (self.stop or self.stalled or k >= self.budget or self.done_total >= self.needed):
            mc, pid = self._select()
            if mc < 2 or self.next_id > TM:
                self.stop = True
            else:
                self.active = True
                self._sel = (mc, pid)
                self.counts[pid] = 0
                a, b = pid >> 16, pid & TM
                ln = self.ln
                s = self.cur[:ln].copy()
                tok = s & TM
                hit = np.zeros(ln, bool)
                if ln >= 2:
                    hit[1:] = ((s[1:] & WS) == 0) & (tok[:-1] == a) & (tok[1:] == b)
                rw = np.zeros(ln, bool)
                rw[:-1] = hit[1:]
                news = s.copy()
                news[rw] = np.uint32(self.next_id) | (s[rw] & WS)
                gnew = self.gn - mc
                limit = ln if self.exact else min(max(gnew - self.off, 0), ln)
                idx = np.flatnonzero(~hit)
                kept_idx = idx[idx < limit]
                kept = news[kept_idx]
                m_r = int(idx.shape[0] - kept_idx.shape[0])
                old, new = _pairs(s), _pairs(kept)
                deltas = {}
                for p in set(old) | set(new):
                    if p == pid:
                        continue
                    d = new.get(p, 0) - old.get(p, 0)
                    if d:
                        deltas[p] = d
                # stale-window superset piece: global [gnew - mc, gnew) of the previous input stream
                w = np.zeros(0, np.uint32)
                if not self.exact:
                    lo, hi = max(gnew - mc, 0), gnew
                    a0, a1 = max(lo, self.poff), min(hi, self.poff + self.pln)
                    if a1 > a0:
                        w = self.oth[a0 - self.poff: a1 - self.poff].copy()
                lst = np.array(sorted(deltas.items()), dtype=np.int64).reshape(-1, 2)
                rec[H_ACTIVE] = 1
                rec[H_L] = lst.shape[0]
                rec[H_KEPT] = kept.shape[0]
                rec[H_M] = m_r
                rec[H_W] = w.shape[0]
                if kept.shape[0]:
                    rec[H_LASTSYM] = kept[-1]
                    rec[H_HASLAST] = 1
                rec[H_SURV] = idx.shape[0]
                rec[H_LN] = ln
                rec[H_MC], rec[H_A], rec[H_B], rec[H_ID] = mc, a, b, self.next_id
                nl = min(lst.shape[0], C)
                if nl:
                    rec[HDR: HDR + 2 * nl] = lst[:nl].astype(np.uint32).reshape(-1)
                nw_ = min(w.shape[0], Cw)
                rec[HDR + 2 * C: HDR + 2 * C + nw_] = w[:nw_]
                self._pending = (news, kept, hit)
        import torch
        send.copy_(torch.from_numpy(rec.view(np.int32)))

    def phase2(self, k, recv, C, Cw):
        if not self.active:
            return
        R = self.world
        rw = HDR + 2 * C + Cw
        recs = recv.cpu().numpy().view(np.uint32).reshape(R, rw)
        hd = recs[:, :HDR]
        assert (hd[:, H_ACTIVE] == 1).all()
        mc, pid = self._sel
        if (hd[:, H_L] > C).any() or (hd[:, H_W] > Cw).any():
            self.counts[pid] = mc            # undo the selection
            self.stalled = True
            self.need = (int(hd[:, H_L].max()), int(hd[:, H_W].max()))
            self.active = False
            return
        assert int(hd[:, H_SURV].sum()) == self.gn - mc
        self.peak = (max(self.peak[0], int(hd[:, H_L].max())), max(self.peak[1], int(hd[:, H_W].max())))
        gnew = self.gn - mc
        m = int(hd[:, H_M].sum())
        pieces = [recs[q, HDR + 2 * C: HDR + 2 * C + hd[q, H_W]] for q in range(R)]
        sup = np.concatenate(pieces) if pieces else np.zeros(0, np.uint32)
        if self.exact:
            m = 0
        win = sup[sup.shape[0] - m:] if m else np.zeros(0, np.uint32)
        kept_q = hd[:, H_KEPT].astype(np.int64)
        owners = np.flatnonzero(kept_q > 0)
        owner = int(owners[-1]) if owners.size else 0
        has_x0 = owners.size > 0
        if m and sum(1 for q in range(R) if hd[q, H_W]) > 1:
            self.events["window_multi_rank"] += 1
        if m and owner != R - 1:
            self.events["owner_not_last"] += 1
        x0 = int(hd[owner, H_LASTSYM]) if has_x0 else 0
        # deltas of every rank + the window's pairs
        for q in range(R):
            L = int(hd[q, H_L])
            lst = recs[q, HDR: HDR + 2 * L].reshape(-1, 2)
            for p, d in lst.tolist():
                d = d - (1 << 32) if d >= (1 << 31) else d
                self.counts[p] = self.counts.get(p, 0) + d
        for j in range(m):
            x = int(win[j])
            if j == 0:
                if not has_x0:
                    continue
                xp = x0
            else:
                xp = int(win[j - 1])
            if not (x & WS) and (xp & TM) and (x & TM):
                p = ((xp & TM) << 16) | (x & TM)
                self.counts[p] = self.counts.get(p, 0) + 1
        a, b = pid >> 16, pid & TM
        self.log.append([a, b, self.next_id, mc])
        self.next_id += 1
        self.done_total += 1
        # local stream: in-place rewrite of the input buffer, compaction into the other one
        news, kept, hit = self._pending
        self.cur[: self.ln] = news
        nl = kept.shape[0]
        self.oth[:nl] = kept
        if self.rank == owner and m:
            self.oth[nl: nl + m] = win
            nl += m
        newlens = [int(kept_q[q]) + (m if q == owner else 0) for q in range(R)]
        assert sum(newlens) == gnew
        self.events["empty_ranks"] = max(self.events["empty_ranks"], sum(1 for x in newlens if x == 0))
        self.cur, self.oth = self.oth, self.cur
        self.poff, self.pln = self.off, self.ln
        self.ln = nl
        self.off = sum(newlens[: self.rank])
        self.gn = gnew
        self.active = False

    def step_end(self):
        need = self.need if self.stalled else self.peak
        return {"merges": self.log, "early_stop": self.stop, "stalled": self.stalled,
                "need_list": need[0], "need_win": need[1]}

    def symbols(self):
        return self.cur[: self.ln].copy()

    # ── consolidation ──
    def global_len(self):
        return self.gn

    def export_state(self):
        """current local stream + the previous input stream (the stale-window source)"""
        return self.cur[: self.ln].copy(), self.oth[: self.pln].copy()


class OracleSingle:
    """The consolidated run on the CPU: the oracle's merge loop (bpe_oracle.train's
    body) continued from a gathered (current, previous) global state."""

    def __init__(self, cur, prev, next_id: int, exact: bool = False):
        n, npv = int(cur.shape[0]), int(prev.shape[0])
        cap = max(n, npv) + 16
        self.cur = np.zeros(cap, np.uint32)
        self.oth = np.zeros(cap, np.uint32)
        self.cur[:n] = cur
        self.oth[:npv] = prev
        self.n = n
        self.nxt = next_id
        self.compaction = "exact" if exact else "reference"

    def step(self, k):
        out = []
        for _ in range(k):
            uniq, counts = O.count_pairs(self.cur[: self.n])
            mc, pid = O.select_best(uniq, counts)
            if mc < 2 or self.nxt > TM:
                return out, True
            a, b = pid >> 16, pid & TM
            self.n, _ = O.merge_step(self.cur, self.oth, self.n, a, b, self.nxt, self.compaction)
            out.append([a, b, self.nxt, mc])
            self.nxt += 1
            self.cur, self.oth = self.oth, self.cur
        return out, False

    def symbols(self):
        return self.cur[: self.n].copy()
