"""Sharded first pass + lexicon hand-over: one rank per GPU.

SURVEY §8(e): the corpus is cut at word starts, so pair counts add up across
pieces (train.wgsl:395; pairs never span a word start), and the merge chain the
reference runs on one device (training-pipeline.js:178-222) is sequential —
every merge's argmax needs the counts after the previous merge.  So the ranks
share the part that is not a chain, the first pass over the corpus:

* every rank turns its piece into symbols, word boundaries and pair counts
  (``gbpe_lexshard_create``), reports its largest count, and builds its word
  lexicon (``gbpe_lexshard_build``): its distinct words, each with its
  multiplicity, plus the occurrence list that keeps its stream order;
* the sum of the ranks' largest counts bounds the first merge's global count,
  which sizes the dense zone (the stream's tail, where the reference compaction
  quirk acts, train.wgsl:605-607 + 698/727): the last ranks keep their part of
  it dense — the tail of one piece and every piece after it;
* the stores and the zone parts go to ONE root, the last rank, which deduplicates
  them into one lexicon, counts the pairs and continues with the single-device
  sector-sparse loop (``gbpe_trainer_create_from_lexicon``) from the first merge;
* the root broadcasts the merge list; on request it sends each rank its slice of
  the word-id map and rebuilds the final stream from every rank's occurrence
  list (``gbpe_trainer_expand``) — the stream itself never sits on one device.

Transport: RCCL (``nccl``) moves device tensors point to point; ``staged`` runs
(gloo; several ranks sharing one GPU in tests and rehearsals) move host copies.
Scalar bookkeeping goes over ``host_group`` (gloo) when given.  The backend is
the C-ABI (``GpuLexBackend``); tests drive the same host loop with a numpy
model of a rank and of the root over gloo (tests/lexshard_model.py).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from . import _lib

BATCH_SIZE = 128
STORE, MUL, OCC, ZONE = _lib.GBPE_LEXSHARD_STORE, _lib.GBPE_LEXSHARD_MUL, _lib.GBPE_LEXSHARD_OCC, _lib.GBPE_LEXSHARD_ZONE


class _Xfer:
    """The few collectives the hand-over needs, over device tensors (RCCL) or
    host copies (gloo)."""

    def __init__(self, dist, staged: bool, host_group=None):
        import torch
        self.torch = torch
        self.dist = dist
        self.staged = staged
        self.group = host_group
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.dev = "cpu" if staged else "cuda"
        self.sdev = "cpu" if (staged or host_group is not None) else "cuda"   # scalars

    def ints(self, vals):
        """all-gather of a short int64 list -> [world, len] numpy."""
        t = self.torch
        x = t.tensor(vals, dtype=t.int64, device=self.sdev)
        if self.world == 1:
            return x.view(1, -1).cpu().numpy()
        outs = [t.empty_like(x) for _ in range(self.world)]
        self.dist.all_gather(outs, x, group=self.group)
        return t.stack(outs).cpu().numpy()

    def bcast_ints(self, vals, root):
        """int64 list from root to every rank (length first)."""
        if self.world == 1:
            return list(vals)
        t = self.torch
        n = t.tensor([len(vals) if self.rank == root else 0], dtype=t.int64, device=self.sdev)
        self.dist.broadcast(n, src=root, group=self.group)
        buf = t.zeros(max(1, int(n.item())), dtype=t.int64, device=self.sdev)
        if self.rank == root and vals:
            buf[: len(vals)] = t.tensor(vals, dtype=t.int64)
        self.dist.broadcast(buf, src=root, group=self.group)
        return buf[: int(n.item())].cpu().tolist()

    def to_root(self, mine, sizes, root):
        """Every rank's byte buffer (``mine``: torch uint8 of ``sizes[rank]``
        bytes) to root, concatenated in rank order (root: one uint8 tensor)."""
        t = self.torch
        if self.rank != root:
            if sizes[self.rank]:
                self.dist.send(mine.contiguous(), dst=root)
            return None
        total = int(sum(sizes))
        out = t.empty(max(1, total), dtype=t.uint8, device=self.dev)
        off = 0
        for q in range(self.world):
            if sizes[q]:
                if q == root:
                    out[off: off + sizes[q]].copy_(mine)
                else:
                    self.dist.recv(out[off: off + sizes[q]], src=q)
            off += int(sizes[q])
        return out[:total]

    def from_root(self, parts, sizes, root):
        """root's ``parts[q]`` (torch uint8) to rank q; returns this rank's."""
        t = self.torch
        if self.rank == root:
            for q in range(self.world):
                if q != root and sizes[q]:
                    self.dist.send(parts[q].contiguous(), dst=q)
            return parts[root]
        buf = t.empty(max(1, int(sizes[self.rank])), dtype=t.uint8, device=self.dev)
        if sizes[self.rank]:
            self.dist.recv(buf, src=root)
        return buf[: int(sizes[self.rank])]


def _debug_knob(key: str, default: int) -> int:
    """GBPE_DEBUG="key=value,..." (the library's test overrides, csrc/common.h)."""
    for kv in os.environ.get("GBPE_DEBUG", "").split(","):
        k, _, v = kv.partition("=")
        if k == key and v:
            return int(v)
    return default


def _ptr(x):
    """(pointer, on_device) of a torch tensor or numpy array."""
    if hasattr(x, "data_ptr"):
        return C.c_void_p(x.data_ptr()), 1 if x.is_cuda else 0
    return x.ctypes.data_as(C.c_void_p), 0


class GpuLexBackend:
    """A rank's lexicon shard and, on the root, the trainer over the gbpe C-ABI."""

    def __init__(self, lib, ctx, target_vocab: int, flags: int = 0, table_log2: int = 0, batch: int = BATCH_SIZE):
        self.lib, self.ctx = lib, ctx
        self.opts = _lib.TrainOpts(target_vocab_size=target_vocab, vocab_size=256, next_token_id=256,
                                   batch_size=batch, flags=flags, table_log2=table_log2)
        self.ls = C.c_void_p()
        self.t = C.c_void_p()
        self.batch = batch
        self._out = (C.c_uint32 * (4 * batch))()

    def _check(self, rc, what):
        _lib.check(rc, self.ctx, what)

    def _info(self):
        i = _lib.LexShardInfo()
        self._check(self.lib.gbpe_lexshard_info_get(self.ls, C.byref(i)), "lexshard_info_get")
        return {f: int(getattr(i, f)) for f, _ in _lib.LexShardInfo._fields_}

    def create(self, piece, n: int, on_device: bool, word_starts=None) -> dict:
        ws = None
        if word_starts is not None:
            self._ws = np.ascontiguousarray(word_starts, dtype=np.uint8)
            ws = self._ws.ctypes.data_as(C.c_void_p)
        self._check(self.lib.gbpe_lexshard_create(self.ctx, piece, n, ws, 1 if on_device else 0, C.byref(self.opts),
                                                  C.byref(self.ls)), "lexshard_create")
        return self._info()

    def build(self, zone_target: int) -> dict:
        self._check(self.lib.gbpe_lexshard_build(self.ls, zone_target), "lexshard_build")
        return self._info()

    def export(self, part: int, nbytes: int, device: str):
        import torch
        buf = torch.empty(max(1, nbytes), dtype=torch.uint8, device=device)
        if nbytes:
            p, d = _ptr(buf)
            self._check(self.lib.gbpe_lexshard_copy(self.ls, part, p, nbytes, d), "lexshard_copy")
        return buf[:nbytes]

    def release(self):
        self._check(self.lib.gbpe_lexshard_release(self.ls), "lexshard_release")

    def remap(self, map_bytes, n_map: int):
        if hasattr(map_bytes, "is_cuda") and map_bytes.is_cuda:
            import torch
            torch.cuda.current_stream().synchronize()   # received on torch's stream; read on the library's
        p, d = _ptr(map_bytes)
        self._check(self.lib.gbpe_lexshard_remap(self.ls, p, n_map, d), "lexshard_remap")

    def root_create(self, stores, muls, zone, store_len: int, zone_len: int, body_len: int, n_entries: int):
        """The root trainer; returns the word-id map (uint8 view of u32) on the inputs' device."""
        import torch
        on_dev = hasattr(stores, "is_cuda") and stores.is_cuda
        if on_dev:
            torch.cuda.current_stream().synchronize()   # received on torch's stream; read on the library's
        mp = torch.empty(max(1, n_entries), dtype=torch.int32, device="cuda" if on_dev else "cpu")
        nm = C.c_uint64()
        a, _ = _ptr(stores)
        b, _ = _ptr(muls)
        z, _ = _ptr(zone)
        m, md = _ptr(mp)
        self._check(self.lib.gbpe_trainer_create_from_lexicon(self.ctx, a, b, store_len, z, zone_len, body_len,
                                                              1 if on_dev else 0, C.byref(self.opts), m, n_entries,
                                                              C.byref(nm), md, C.byref(self.t)),
                    "trainer_create_from_lexicon")
        if int(nm.value) != n_entries:
            raise RuntimeError(f"lexicon hand-over: {nm.value} map entries for {n_entries} store entries")
        return mp[:n_entries].view(torch.uint8)

    def root_step(self, k: int):
        nd, es = C.c_uint32(), C.c_uint32()
        self._check(self.lib.gbpe_trainer_step(self.t, min(k, self.batch), self._out, C.byref(nd), C.byref(es)),
                    "root step")
        return [list(self._out[4 * i: 4 * i + 4]) for i in range(nd.value)], bool(es.value)

    def root_expand(self, prefix, n_prefix: int) -> np.ndarray:
        import torch
        if hasattr(prefix, "is_cuda") and prefix.is_cuda:
            torch.cuda.current_stream().synchronize()
        n = C.c_uint64()
        self._check(self.lib.gbpe_trainer_expand(self.t, None, 0, 0, None, 0, C.byref(n), 0), "expand")
        out = np.zeros(max(1, n.value), dtype=np.uint32)
        p, d = _ptr(prefix)
        got = C.c_uint64()
        self._check(self.lib.gbpe_trainer_expand(self.t, p, n_prefix, d, out.ctypes.data_as(C.c_void_p), n.value,
                                                 C.byref(got), 0), "expand")
        return out[: got.value]

    def root_stats(self):
        st = _lib.TrainerStats()
        self.lib.gbpe_trainer_stats_get(self.t, C.byref(st))
        return st

    def close(self):
        if self.t:
            self.lib.gbpe_trainer_destroy(self.t)
            self.t = C.c_void_p()
        if self.ls:
            self.lib.gbpe_lexshard_destroy(self.ls)
            self.ls = C.c_void_p()


class LexShardTrainer:
    """Host loop of the hand-over: ``train(piece)`` on every rank returns the
    global merge list on every rank.  The root is the last rank (it holds the
    zone); ``staged`` moves host copies (gloo), else device tensors (RCCL)."""

    def __init__(self, backend, dist, staged: bool = False, host_group=None, sp_zt: int | None = None):
        self.b = backend
        self.x = _Xfer(dist, staged, host_group)
        self.rank, self.world = self.x.rank, self.x.world
        self.root = self.world - 1
        self.staged = staged
        self.sp_zt = max(3, sp_zt if sp_zt is not None else _debug_knob("zt", 5))
        self.timing = {}
        self.shapes = None
        self.map = None
        self.root_stats = None

    def _agree(self, failed: bool, err, what: str):
        """Every rank learns whether any rank failed since the last exchange and
        raises alike (a rank that left early would leave its peers blocked in the
        next collective)."""
        bad = self.x.ints([1 if failed else 0])[:, 0]
        if bad.any():
            if err is not None:
                raise err
            raise RuntimeError(f"lexicon hand-over: rank(s) {np.flatnonzero(bad).tolist()} failed in {what}")

    def zone_targets(self, lens, ub: int):
        """Per-rank zone targets: the zone is the stream's last zt symbols (the zone
        rule's target for a first count <= ub, trainer.h sp_enter), which may span
        the tails of several pieces; a rank whose piece lies wholly inside it keeps
        the whole piece dense (target = its length), the rank where it begins keeps
        its tail from the last word start at or before the zone's start."""
        zt = max(self.sp_zt * ub, 2 * ub) + 64
        N = int(np.sum(lens))
        if zt + 2 >= N:
            raise RuntimeError(f"lexicon hand-over: a zone of {zt} symbols does not fit the {N}-symbol stream")
        G = N - zt
        offs = np.concatenate([[0], np.cumsum(lens)])
        out = []
        for q in range(len(lens)):
            a, b = int(offs[q]), int(offs[q + 1])
            out.append(0 if b <= G else (b - a if a >= G else b - G))
        return out

    def first_pass(self, piece, n: int, on_device: bool, word_starts=None):
        """Symbols, counts and the word lexicon of this rank's piece; stores and
        zone parts to the root.  Returns the root's inputs there, None elsewhere."""
        t0 = time.perf_counter()
        info, err = None, None
        try:
            info = self.b.create(piece, n, on_device, word_starts)
        except Exception as e:  # noqa: BLE001 — every rank raises below
            err = e
        g = self.x.ints([info["top_count"], info["symbols"], 0] if info else [0, 0, 1])
        if g[:, 2].any():
            if err is not None:
                raise err
            raise RuntimeError(f"lexicon hand-over: rank(s) {np.flatnonzero(g[:, 2]).tolist()} failed in create")
        ub = int(g[:, 0].sum())   # >= the first merge's global count
        zts = self.zone_targets(g[:, 1], ub)
        self.timing["create_s"] = time.perf_counter() - t0
        try:
            info = self.b.build(zts[self.rank])
        except Exception as e:  # noqa: BLE001
            err, info = e, None
        sh = self.x.ints([info["store_symbols"], info["entries"], info["words"], info["body"], info["zone"],
                          info["symbols"], 0] if info else [0] * 6 + [1])
        if sh[:, 6].any():
            if err is not None:
                raise err
            raise RuntimeError(f"lexicon hand-over: rank(s) {np.flatnonzero(sh[:, 6]).tolist()} failed in build")
        self.shapes = sh[:, :6]
        self.timing["build_s"] = time.perf_counter() - t0
        bps = info["bytes_per_symbol"]
        store = mul = zone = None
        try:
            T = info["store_symbols"]
            store = self.b.export(STORE, T * bps, self.x.dev)
            mul = self.b.export(MUL, T * 4, self.x.dev)
            zone = self.b.export(ZONE, info["zone"] * bps, self.x.dev)
            self.b.release()   # the piece's stream and counts are no longer needed
        except Exception as e:  # noqa: BLE001
            err = e
        self._agree(err is not None, err, "export")
        stores = self.x.to_root(store, [int(v) * bps for v in sh[:, 0]], self.root)
        muls = self.x.to_root(mul, [int(v) * 4 for v in sh[:, 0]], self.root)
        zones = self.x.to_root(zone, [int(v) * bps for v in sh[:, 4]], self.root)   # in rank order: the stream's tail
        self.timing["exchange_s"] = time.perf_counter() - t0
        return (stores, muls, zones) if self.rank == self.root else None

    def train(self, piece, n: int, on_device: bool, target_vocab: int, word_starts=None, batch: int = BATCH_SIZE,
              on_progress=None):
        """The whole run; every rank returns (merges, early_stop)."""
        t0 = time.perf_counter()
        got = self.first_pass(piece, n, on_device, word_starts)
        merges, early, err = [], False, None
        if self.rank == self.root:
            try:
                sh = self.shapes
                t1 = time.perf_counter()
                self.map = self.b.root_create(*got, int(sh[:, 0].sum()), int(sh[:, 4].sum()), int(sh[:, 3].sum()),
                                              int(sh[:, 1].sum()))
                del got
                t2 = time.perf_counter()
                self.timing["root_create_s"] = t2 - t1
                needed = target_vocab - 256
                while len(merges) < needed:
                    got_m, early = self.b.root_step(min(batch, needed - len(merges)))
                    merges += got_m
                    if on_progress:
                        on_progress(len(merges), needed)
                    if early or not got_m:
                        break
                self.timing["loop_s"] = time.perf_counter() - t2
                self.root_stats = self.b.root_stats()
            except Exception as e:  # noqa: BLE001 — reported to every rank below
                err = e
        flat = ([1 if early else 0] + [int(v) for m in merges for v in m]) if err is None else [-1]
        flat = self.x.bcast_ints(flat, self.root)
        if err is not None:
            raise err
        if flat[0] < 0:
            raise RuntimeError(f"lexicon hand-over: the root rank {self.root} failed")
        self.timing["total_s"] = time.perf_counter() - t0
        return [flat[1 + 4 * i: 5 + 4 * i] for i in range((len(flat) - 1) // 4)], bool(flat[0])

    def final_stream(self):
        """The final stream (u32 reference layout) on the root, None elsewhere.
        Collective: every rank's occurrence list is remapped to the root's word ids
        and gathered to the root, which expands them with its store and zone."""
        sh = self.shapes
        sizes = [int(v) * 4 for v in sh[:, 1]]
        parts = None
        if self.rank == self.root:
            offs = np.concatenate([[0], np.cumsum(sizes)])
            parts = [self.map[int(offs[q]): int(offs[q + 1])] for q in range(self.world)]
        mine = self.x.from_root(parts, sizes, self.root)
        occ, err = None, None
        try:
            self.b.remap(mine, int(sh[self.rank, 1]))
            occ = self.b.export(OCC, int(sh[self.rank, 2]) * 4, self.x.dev)
        except Exception as e:  # noqa: BLE001
            err = e
        self._agree(err is not None, err, "remap / occurrence export")
        allocc = self.x.to_root(occ, [int(v) * 4 for v in sh[:, 2]], self.root)
        if self.rank != self.root:
            return None
        return self.b.root_expand(allocc, int(sh[:, 2].sum()))


def pieces_at_word_starts(dist, shard: bytes, word_boundary, host_group=None, halo: int = 1 << 16) -> bytes:
    """Rank r's piece of a corpus given as R consecutive shards (C4: 8 x 1 GiB,
    seed 5 + r): shard r from the first position of the CONCATENATED stream that
    is a word start under the reference heuristic (train.wgsl:111-186 reads the
    byte before it: the previous shard's last byte), extended by the next shard's
    head up to that shard's first word start.  The pieces concatenate to the
    shards' concatenation, and each starts a word.  ``word_boundary(bytes) ->
    uint8 mask`` is the heuristic (gbpe_word_boundary on the device)."""
    import torch
    R, r = dist.get_world_size(), dist.get_rank()
    H = halo
    if R > 1:   # one halo length on every rank (the all-gather needs equal sizes)
        ln = torch.tensor([len(shard)], dtype=torch.int64)
        lns = [torch.empty_like(ln) for _ in range(R)]
        dist.all_gather(lns, ln, group=host_group)
        H = min(halo, min(int(v.item()) for v in lns))
    H = min(H, len(shard))
    head = np.zeros(H + 1, dtype=np.uint8)
    head[0] = shard[-1]                       # the last byte: the next shard's boundary reads it
    head[1:] = np.frombuffer(shard[:H], dtype=np.uint8)
    mine = torch.from_numpy(head)
    if R > 1:
        outs = [torch.empty_like(mine) for _ in range(R)]
        dist.all_gather(outs, mine, group=host_group)
        allh = torch.stack(outs).numpy()
    else:
        allh = head[None, :]

    def head_len(q):   # bytes at the start of shard q that continue shard q-1's last word
        if q == 0:
            return 0
        ws = np.asarray(word_boundary(np.concatenate([allh[q - 1, :1], allh[q, 1:]]).tobytes()), dtype=np.uint8)
        st = np.flatnonzero(ws[1:])
        if st.shape[0] == 0:
            raise RuntimeError(f"shard {q}: no word start in its first {H} bytes")
        return int(st[0])

    piece = shard[head_len(r):]
    if r + 1 < R:
        piece += allh[r + 1, 1: 1 + head_len(r + 1)].tobytes()
    return piece


def device_word_boundary(lib, ctx):
    """gbpe_word_boundary (train.wgsl:87-186 on the device) as a bytes -> mask function."""
    def f(b: bytes) -> np.ndarray:
        ws = np.zeros(len(b), dtype=np.uint8)
        _lib.check(lib.gbpe_word_boundary(ctx, b, len(b), ws.ctypes.data_as(C.c_void_p)), ctx, "word_boundary")
        return ws
    return f
