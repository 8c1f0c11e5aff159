"""numpy model of the lexicon hand-over backend — TEST INFRASTRUCTURE ONLY.

Implements the backend interface of ``gpubpe.lexshard.LexShardTrainer`` with
plain numpy and the oracle, so the host loop (collectives, rank order, the
word-id map, remapping, the final-stream expansion) runs on the CPU over gloo:

* a rank (``create`` / ``build``): the piece's symbols (u32 reference layout,
  bit 16 = word start) and pair counts, the zone start (the last position at or
  before n - zt that no counted pair spans), its distinct words in first-seen
  order with their multiplicities, the store (each word + a 0 separator), and
  the occurrence list — what csrc/train_lexshard.hip's ls_build produces (in
  another word-id order: the C build numbers words by hash slot);
* the root (``root_create`` / ``root_step`` / ``root_expand``): the weighted
  deduplication of the concatenated stores, then the oracle's merge loop over an
  EQUIVALENT stream — every distinct word repeated by its multiplicity, each copy
  followed by a 0, then the zone.  No counted pair spans a 0 and every copy of a
  word merges alike, so the pair counts, and with the zone holding the stale
  window of every merge (the zone rule), the merges, are the real stream's.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import bpe_oracle as O  # noqa: E402

WS, TM = O.WORD_START_BIT, O.TOKEN_MASK
LIT = 0x80000000


def _starts(s: np.ndarray) -> np.ndarray:
    """positions no counted pair can span: a word start, or token 0 on either side"""
    st = np.zeros(s.shape[0], dtype=bool)
    if s.shape[0]:
        st[0] = True
        tok = s & TM
        st[1:] = ((s[1:] & WS) != 0) | (tok[1:] == 0) | (tok[:-1] == 0)
    return st


def _words(s: np.ndarray):
    b = np.flatnonzero(_starts(s)).tolist() + [s.shape[0]]
    return [s[b[i]: b[i + 1]] for i in range(len(b) - 1)]


class ModelLexBackend:
    def __init__(self, exact: bool = False):
        self.exact = exact

    # ── rank ──
    def create(self, piece, n, on_device, word_starts=None):
        assert not on_device
        self.s = O.prepare_symbols(bytes(piece), word_starts)
        u, c = O.count_pairs(self.s)
        self.top = int(c.max()) if c.size else 0
        return self._info(built=False)

    def _info(self, built=True):
        n = int(self.s.shape[0])
        return {"symbols": n, "body": self.Zs if built else n, "zone": n - self.Zs if built else 0,
                "store_symbols": int(self.store.shape[0]) if built else 0, "entries": len(self.uids) if built else 0,
                "words": len(self.occ) if built else 0, "top_count": self.top, "bytes_per_symbol": 4}

    def build(self, zone_target):
        s, n = self.s, int(self.s.shape[0])
        Zs = n
        if zone_target >= n:   # the whole piece lies inside the zone
            Zs = 0
        elif zone_target:
            st = np.flatnonzero(_starts(s)[: n - zone_target + 1])
            Zs = int(st[-1])
        self.Zs = Zs
        self.uids, mult, self.occ = {}, [], []
        for w in _words(s[:Zs]):
            if (int(w[0]) & TM) == 0:
                self.occ.append(LIT | int(w[0]))
                continue
            k = w.tobytes()
            if k not in self.uids:
                self.uids[k] = len(self.uids)
                mult.append(0)
            u = self.uids[k]
            mult[u] += 1
            self.occ.append(u)
        words = [np.frombuffer(k, dtype=np.uint32) for k in self.uids]
        self.store = np.concatenate([np.append(w, 0).astype(np.uint32) for w in words]) if words else \
            np.zeros(0, np.uint32)
        self.mul = np.concatenate([np.full(w.shape[0] + 1, m, np.uint32) for w, m in zip(words, mult)]) if words else \
            np.zeros(0, np.uint32)
        if words:   # separators carry multiplicity 0
            ends = np.cumsum([w.shape[0] + 1 for w in words]) - 1
            self.mul[ends] = 0
        self.zone = s[Zs:].copy()
        self.occ = np.array(self.occ, dtype=np.uint32)
        return self._info()

    def export(self, part, nbytes, device):
        import torch
        a = {0: self.store, 1: self.mul, 2: self.occ, 3: self.zone}[part]
        b = torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.uint8).copy())
        assert b.numel() == nbytes
        return b

    def release(self):
        pass

    def remap(self, map_bytes, n_map):
        mp = map_bytes.numpy().view(np.uint32)
        assert mp.shape[0] == n_map
        lit = (self.occ & LIT) != 0
        self.occ = np.where(lit, self.occ, mp[np.where(lit, 0, self.occ)]).astype(np.uint32)

    # ── root ──
    def root_create(self, stores, muls, zone, store_len, zone_len, body_len, n_entries):
        import torch
        st = stores.numpy().view(np.uint32)
        mu = muls.numpy().view(np.uint32)
        zn = zone.numpy().view(np.uint32)
        assert st.shape[0] == store_len and zn.shape[0] == zone_len
        ends = np.flatnonzero(st == 0)
        starts = np.concatenate([[0], ends[:-1] + 1])
        assert ends.shape[0] == n_entries
        self.gid, self.gmult, self.gwords, mp = {}, [], [], []
        for a, e in zip(starts, ends):
            w = st[a:e]
            k = w.tobytes()
            if k not in self.gid:
                self.gid[k] = len(self.gid)
                self.gmult.append(0)
                self.gwords.append(w.copy())
            g = self.gid[k]
            self.gmult[g] += int(mu[a])
            mp.append(g)
        assert sum(w.shape[0] * m for w, m in zip(self.gwords, self.gmult)) == body_len
        # the equivalent stream: every distinct word x its multiplicity, each copy + 0, then the zone
        parts = [np.tile(np.append(w, 0).astype(np.uint32), m) for w, m in zip(self.gwords, self.gmult)]
        self.nsep = sum(self.gmult)
        cur = np.concatenate(parts + [zn]).astype(np.uint32)
        self.single = OracleSingle(cur, np.zeros(0, np.uint32), 256, self.exact)
        return torch.from_numpy(np.array(mp, dtype=np.uint32).view(np.uint8).copy())

    def root_step(self, k):
        return self.single.step(k)

    def root_expand(self, prefix, n_prefix):
        occ = prefix.numpy().view(np.uint32)
        assert occ.shape[0] == n_prefix
        fin = self.single.symbols()
        zpos = np.flatnonzero(fin == 0)
        cut = int(zpos[self.nsep - 1]) + 1 if self.nsep else 0   # every separator survives; windows land in the zone
        body, zone = fin[:cut], fin[cut:]
        final_word, i = [], 0
        for w, m in zip(self.gwords, self.gmult):   # the first copy of every word
            j = i
            while body[j] != 0:
                j += 1
            final_word.append(body[i:j])
            i = j + 1 + 0
            for _ in range(m - 1):                  # skip the other copies (+ their separators)
                while body[i] != 0:
                    i += 1
                i += 1
        out = [final_word[o] if not (o & LIT) else np.array([o & ~LIT], np.uint32) for o in occ.tolist()]
        return np.concatenate(out + [zone]).astype(np.uint32)

    def root_stats(self):
        return None

    def close(self):
        pass


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
