"""Sharded BPE training: one process per GPU, bit-exact global merges.

SURVEY §8(e): the corpus is cut at word starts, so pair counts are additive
across shards (train.wgsl:395; pairs never cross a word start).  Every merge
still needs a global argmax, and the reference's compaction quirk
(train.wgsl:605-607 + 698/727) acts on the *global* stream end.  Each rank
therefore keeps a replica of the global pair-count table, and every merge is
one fixed-size all-gather of a per-rank *exchange record*:

    header (HDR u32) | count deltas (C x {pid, delta}) | window piece (Cw u32)

* phase 1 (per rank, device): select on the replica (identical on all ranks),
  find the merge sites in the local stream, aggregate the local count deltas,
  and copy this rank's piece of the stale-window superset
  ``[n' - mc, n')`` (global positions; the previous merge's input stream, the
  ping-pong buffer the reference reads stale symbols from);
* one all-gather of the records (RCCL over xGMI on MI355X; gloo on CPU);
* phase 2 (per rank, device, identical decisions on every rank): apply every
  rank's deltas to the replica, cut the stale window (last ``m`` symbols of the
  superset) and add its pairs, compact the local stream; the last rank that
  kept any survivor appends the window, so the global stream stays the
  concatenation of the rank streams in rank order.

Capacities ``C``/``Cw`` are fixed per step, so no host synchronisation happens
inside a 128-merge step.  A merge whose record does not fit stalls on every
rank (its selection is undone), the step ends early, and the host grows the
capacity from the needs recorded in the gathered headers and continues — the
merge list is unaffected.

Consolidation (``train(..., consolidate_below=N)``): once the global stream is
at most N symbols, merges are latency-bound and the per-merge exchange costs
more than the merge.  The ranks then export their current and previous local
streams, ``root`` gathers them (concatenated in rank order they ARE the global
streams, the previous one included, so the compaction quirk's stale window
reads the same symbols), continues on one device (``GpuSingleBackend``:
gbpe_trainer_create_from_state, the single-GPU loop with its lexicon / sparse
policy), and broadcasts the merge list at the end.

The backend is the C-ABI trainer (``GpuShardBackend``); tests drive the same
orchestration with a numpy model of one rank over gloo.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

# exchange-record header words (mirrored by csrc/train.hip)
H_ACTIVE, H_L, H_KEPT, H_M, H_W, H_LASTSYM, H_HASLAST, H_SURV, H_LN, H_MC, H_A, H_B, H_ID, H_DFULL = range(14)
HDR = 16
BATCH_SIZE = 128


def record_words(cap_list: int, cap_win: int) -> int:
    return HDR + 2 * cap_list + cap_win


def _pow2_at_least(x: int, lo: int) -> int:
    v = lo
    while v < x:
        v <<= 1
    return v


class ShardedTrainer:
    """Host loop over a shard backend (trainer.js:225-335 per rank).

    ``dist`` is ``torch.distributed`` (initialised); ``staged`` copies device
    records through host memory (gloo with device buffers, e.g. several ranks
    sharing one GPU in tests)."""

    def __init__(self, backend, dist, device="cpu", staged: bool = False, cap_list: int = 1 << 14,
                 cap_win: int = 1 << 12):
        import torch
        self.torch = torch
        self.b = backend
        self.dist = dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.device = device
        self.staged = staged
        self.C = cap_list
        self.Cw = cap_win
        self.min_list, self.min_win = min(cap_list, 1 << 12), min(cap_win, 1 << 10)
        self.adaptive = True
        self.stalls = 0
        self._bufs = None

    # ── collectives ──
    def _all_gather(self, send):
        torch = self.torch
        out = torch.empty(self.world * send.numel(), dtype=send.dtype, device=send.device)
        if self.staged and send.device.type != "cpu":
            hs = send.cpu()
            ho = torch.empty(self.world * send.numel(), dtype=send.dtype)
            self.dist.all_gather_into_tensor(ho, hs)
            out.copy_(ho)
        else:
            self.dist.all_gather_into_tensor(out, send)
        return out

    def _gather_ints(self, vals):
        torch = self.torch
        t = torch.tensor(vals, dtype=torch.int64, device=self.device)
        return self._all_gather(t).view(self.world, len(vals)).cpu().numpy()

    def setup(self):
        """Global layout + the initial global pair counts (one variable-size exchange)."""
        torch = self.torch
        lens = self._gather_ints([self.b.local_len()])[:, 0]
        self.b.set_layout([int(x) for x in lens])
        pairs = self.b.export_counts(self.device)          # int32 [P, 2] (pid, count)
        P = int(pairs.shape[0])
        Ps = self._gather_ints([P])[:, 0]
        pmax = max(1, int(Ps.max()))
        send = torch.zeros(pmax * 2, dtype=torch.int32, device=self.device)
        if P:
            send[: 2 * P] = pairs.reshape(-1)
        allp = self._all_gather(send).view(self.world, pmax * 2)
        self.b.import_counts(allp, [int(x) for x in Ps], pmax)

    def _buffers(self):
        torch = self.torch
        rw = record_words(self.C, self.Cw)
        if self._bufs is None or self._bufs[0].numel() != rw:
            send = torch.zeros(rw, dtype=torch.int32, device=self.device)
            recv = torch.zeros(self.world * rw, dtype=torch.int32, device=self.device)
            self._bufs = (send, recv)
        return self._bufs

    def attach_native_comm(self, comm=None):
        """Let the backend run whole steps natively (RCCL all-gather on its own
        stream).  The 128-byte communicator id travels over ``dist``.  Pass a
        communicator from an earlier trainer (``backend.comm``) to reuse it:
        creating one costs far more than a step."""
        if comm is not None:
            self.b.comm, self.b.owns_comm = comm, False
            self.native = True
            return comm
        torch = self.torch
        idt = torch.zeros(128, dtype=torch.uint8, device=self.device)
        if self.rank == 0:
            idt.copy_(torch.from_numpy(self.b.comm_unique_id()))
        if self.staged and idt.device.type != "cpu":
            h = idt.cpu()
            self.dist.broadcast(h, src=0)
            idt = h
        else:
            self.dist.broadcast(idt, src=0)
        self.b.comm_create(idt.cpu().numpy())
        self.native = True
        return self.b.comm

    native = False

    def step(self, max_merges: int = BATCH_SIZE):
        """Up to ``max_merges`` global merges. Returns (merges, early_stop)."""
        b = self.b
        if self.native:
            res = b.step_comm(max_merges, self.C, self.Cw)
        else:
            b.step_begin(max_merges)
            send, recv = self._buffers()
            for k in range(max_merges):
                b.phase1(k, send, self.C, self.Cw)
                if self.staged or send.device.type == "cpu":
                    out = self._all_gather(send)
                else:
                    self.dist.all_gather_into_tensor(recv, send)
                    out = recv
                b.phase2(k, out, self.C, self.Cw)
            res = b.step_end()
        if res["stalled"]:
            self.stalls += 1
            self.C = _pow2_at_least(2 * res["need_list"], self.C)
            self.Cw = _pow2_at_least(2 * res["need_win"], self.Cw)
        elif res["merges"] and self.adaptive:
            # shrink towards 2x this step's largest record (merges get rarer; the
            # all-gather moves the full capacity every merge); identical on all ranks
            self.C = min(self.C, _pow2_at_least(2 * res["need_list"], self.min_list))
            self.Cw = min(self.Cw, _pow2_at_least(2 * res["need_win"], self.min_win))
        return res["merges"], res["early_stop"]

    def train(self, target_vocab_size: int, vocab_size: int = 256, batch: int = BATCH_SIZE, on_progress=None,
              consolidate_below: int | None = None, make_single=None, root: int = 0):
        """Merges until the target (every rank returns the same list).  With
        ``consolidate_below`` the run moves to ``root`` once the global stream is
        at most that many symbols: ``make_single(cur, prev, next_id)`` builds the
        single-device backend there (``step(k) -> (merges, early_stop)``)."""
        needed = target_vocab_size - vocab_size
        merges = []
        early = False
        self.consolidated_at = None
        while len(merges) < needed:
            if consolidate_below is not None and self.b.global_len() <= consolidate_below:
                return self._finish_on_one(merges, needed, vocab_size, batch, on_progress, make_single, root)
            got, early = self.step(min(batch, needed - len(merges)))
            merges += got
            if on_progress:
                on_progress(len(merges), needed, got)
            if early:
                break
        return merges, early

    # ── consolidation ──
    def _bcast_ints(self, vals, root):
        """int64 list from root to every rank (length first)."""
        torch = self.torch
        dev = "cpu" if self.staged else self.device
        n = torch.tensor([len(vals) if self.rank == root else 0], dtype=torch.int64, device=dev)
        self.dist.broadcast(n, src=root)
        buf = torch.zeros(max(1, int(n.item())), dtype=torch.int64, device=dev)
        if self.rank == root and vals:
            buf[: len(vals)] = torch.tensor(vals, dtype=torch.int64)
        self.dist.broadcast(buf, src=root)
        return buf[: int(n.item())].cpu().tolist()

    def consolidate(self, make_single, next_id: int, root: int = 0):
        """Gather the global (current, previous) streams onto ``root`` and return
        ``make_single(cur, prev, next_id)`` there, None on the other ranks."""
        torch = self.torch
        dev = "cpu" if self.staged else self.device
        on_dev = getattr(self.b, "device_state", False) and dev != "cpu"
        if on_dev:   # HBM to HBM: export into the send buffer, gather over RCCL, concatenate on the device
            n, npv = self.b.state_lens()
            lens = self._gather_ints([n, npv])
            cap = max(1, int(lens.max()))
            send = torch.zeros(2 * cap, dtype=torch.int32, device=dev)
            # the zero fill runs on torch's stream, the export on the library's: order them
            torch.cuda.current_stream().synchronize()
            self.b.export_state_device(send.data_ptr(), send.data_ptr() + 4 * cap, cap, cap)   # (synchronous)
        else:
            cur, prev = self.b.export_state()
            lens = self._gather_ints([int(cur.shape[0]), int(prev.shape[0])])
            cap = max(1, int(lens.max()))
            send = torch.zeros(2 * cap, dtype=torch.int32, device=dev)
            if cur.shape[0]:
                send[: cur.shape[0]] = torch.from_numpy(cur.view(np.int32)).to(dev)
            if prev.shape[0]:
                send[cap: cap + prev.shape[0]] = torch.from_numpy(prev.view(np.int32)).to(dev)
        if self.world == 1:
            parts = [send]
        else:   # all-gather (every backend offers it; gather is not exercised over RCCL)
            allp = self._all_gather(send).view(self.world, 2 * cap)
            parts = [allp[q] for q in range(self.world)]
        if self.rank != root:
            return None
        if on_dev:
            gcur = torch.cat([parts[q][: lens[q, 0]] for q in range(self.world)])
            gprev = torch.cat([parts[q][cap: cap + lens[q, 1]] for q in range(self.world)])
            del parts, send
            torch.cuda.current_stream().synchronize()   # the import reads them on the library's stream
            return make_single(gcur, gprev, next_id)
        host = [p.cpu().numpy().view(np.uint32) for p in parts]
        gcur = np.concatenate([host[q][: lens[q, 0]] for q in range(self.world)])
        gprev = np.concatenate([host[q][cap: cap + lens[q, 1]] for q in range(self.world)])
        return make_single(gcur, gprev, next_id)

    def _finish_on_one(self, merges, needed, vocab_size, batch, on_progress, make_single, root):
        """Root continues alone; every rank then receives the merge list.  A failure
        on root (make_single, a step) is broadcast as status -1, so the other ranks
        raise instead of waiting in the broadcast forever; root re-raises it."""
        self.consolidated_at = len(merges)
        early = False
        flat = []
        err = None
        try:
            single = self.consolidate(make_single, vocab_size + len(merges), root)
            if self.rank == root:
                self.single = single
                while len(merges) < needed:
                    got, early = single.step(min(batch, needed - len(merges)))
                    merges = merges + [list(m) for m in got]
                    if on_progress:
                        on_progress(len(merges), needed, got)
                    if early or not got:
                        break
                flat = [1 if early else 0] + [int(x) for m in merges for x in m]
        except Exception as e:  # noqa: BLE001 — reported to every rank below
            if self.rank != root:
                raise
            err, flat = e, [-1]
        flat = self._bcast_ints(flat, root)
        if err is not None:
            raise err
        if flat[0] < 0:
            raise RuntimeError(f"consolidated training failed on root rank {root}")
        early = bool(flat[0])
        merges = [flat[1 + 4 * i: 5 + 4 * i] for i in range((len(flat) - 1) // 4)]
        return merges, early

    single = None


class GpuShardBackend:
    """One rank's trainer over the gpubpe C-ABI (gbpe_shard_* entry points)."""

    def __init__(self, lib, ctx, data, word_starts, rank: int, world: int, target_vocab: int,
                 exact: bool = False, input_on_device: bool = False, n: int | None = None,
                 table_log2: int = 0, cap_extra: int = 0, stream=None, flags: int = 0):
        from . import _lib
        self.lib, self.ctx, self._lib = lib, ctx, _lib
        if stream is not None:   # run on the caller's stream (torch's), so its collectives and copies are ordered
            _lib.check(lib.gbpe_ctx_set_stream(ctx, C.c_void_p(stream)), ctx, "gbpe_ctx_set_stream")
        flags |= _lib.GBPE_TRAIN_EXACT_COMPACTION if exact else 0
        self.opts = _lib.TrainOpts(target_vocab_size=target_vocab, vocab_size=256, next_token_id=256,
                                   batch_size=BATCH_SIZE, flags=flags, table_log2=table_log2)
        t = C.c_void_p()
        if input_on_device:
            ptr, nn = data, n
        else:
            buf = bytes(data)
            ptr, nn = C.create_string_buffer(buf, len(buf)), len(buf)
        self._keep = ptr
        ws = None
        if word_starts is not None:
            wsb = np.ascontiguousarray(np.asarray(word_starts, dtype=np.uint8))
            ws = wsb.ctypes.data_as(C.c_void_p)
            self._ws_keep = wsb
        _lib.check(lib.gbpe_shard_create(ctx, ptr, nn, ws, 1 if input_on_device else 0, C.byref(self.opts),
                                         rank, world, cap_extra, C.byref(t)), ctx, "gbpe_shard_create")
        self.t = t
        self.rank, self.world = rank, world
        self._out = (C.c_uint32 * (4 * BATCH_SIZE))()

    def local_len(self) -> int:
        n = C.c_uint64()
        self._lib.check(self.lib.gbpe_shard_local_len(self.t, C.byref(n)), self.ctx, "local_len")
        return int(n.value)

    def global_len(self) -> int:
        n = C.c_uint64()
        self._lib.check(self.lib.gbpe_shard_global_len(self.t, C.byref(n)), self.ctx, "global_len")
        return int(n.value)

    def export_state(self):
        return export_state(self.lib, self.ctx, self.t)

    device_state = True   # the hand-over can stay in HBM (RCCL gather of device buffers)

    def state_lens(self):
        return state_lens(self.lib, self.ctx, self.t)

    def export_state_device(self, cur_ptr, prev_ptr, cap_cur, cap_prev):
        return export_state_device(self.lib, self.ctx, self.t, cur_ptr, prev_ptr, cap_cur, cap_prev)

    def set_layout(self, lens):
        arr = (C.c_uint64 * len(lens))(*lens)
        self._lib.check(self.lib.gbpe_shard_set_layout(self.t, arr, len(lens)), self.ctx, "set_layout")

    def export_counts(self, device):
        import torch
        P = C.c_uint64()
        self._lib.check(self.lib.gbpe_shard_export_counts(self.t, None, 0, C.byref(P)), self.ctx, "export")
        out = torch.zeros((max(1, P.value), 2), dtype=torch.int32, device=device)
        self._lib.check(self.lib.gbpe_shard_export_counts(self.t, C.c_void_p(out.data_ptr()), P.value, C.byref(P)),
                        self.ctx, "export")
        return out[: P.value]

    def import_counts(self, allp, counts, pmax):
        arr = (C.c_uint64 * len(counts))(*counts)
        self._lib.check(self.lib.gbpe_shard_import_counts(self.t, C.c_void_p(allp.data_ptr()), arr, len(counts),
                                                          pmax), self.ctx, "import")

    def step_begin(self, max_merges):
        self._lib.check(self.lib.gbpe_shard_step_begin(self.t, max_merges), self.ctx, "step_begin")

    def phase1(self, k, send, cap_list, cap_win):
        self._lib.check(self.lib.gbpe_shard_phase1(self.t, k, C.c_void_p(send.data_ptr()), cap_list, cap_win),
                        self.ctx, "phase1")

    def phase2(self, k, recv, cap_list, cap_win):
        self._lib.check(self.lib.gbpe_shard_phase2(self.t, k, C.c_void_p(recv.data_ptr()), cap_list, cap_win),
                        self.ctx, "phase2")

    def step_end(self):
        nd, es, st, nl, nwn = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._lib.check(self.lib.gbpe_shard_step_end(self.t, self._out, C.byref(nd), C.byref(es), C.byref(st),
                                                     C.byref(nl), C.byref(nwn)), self.ctx, "step_end")
        merges = [list(self._out[4 * i: 4 * i + 4]) for i in range(nd.value)]
        return {"merges": merges, "early_stop": bool(es.value), "stalled": bool(st.value),
                "need_list": int(nl.value), "need_win": int(nwn.value)}

    # ── native exchange (gbpe_shard_step_comm) ──
    comm = None
    owns_comm = True

    def comm_unique_id(self):
        buf = (C.c_uint8 * 128)()
        rc = self.lib.gbpe_comm_unique_id(buf, 128)
        if rc != 0:
            raise self._lib.GpuBpeError(rc, "gbpe_comm_unique_id failed (RCCL unavailable)")
        return np.frombuffer(bytes(buf), dtype=np.uint8).copy()

    def comm_create(self, uid):
        arr = (C.c_uint8 * 128)(*[int(x) for x in uid])
        c = C.c_void_p()
        self._lib.check(self.lib.gbpe_comm_create(self.ctx, arr, 128, self.rank, self.world, C.byref(c)), self.ctx,
                        "gbpe_comm_create")
        self.comm = c

    def step_comm(self, max_merges, cap_list, cap_win):
        nd, es, st, nl, nwn = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._lib.check(self.lib.gbpe_shard_step_comm(self.t, self.comm, max_merges, cap_list, cap_win, self._out,
                                                      C.byref(nd), C.byref(es), C.byref(st), C.byref(nl),
                                                      C.byref(nwn)), self.ctx, "gbpe_shard_step_comm")
        merges = [list(self._out[4 * i: 4 * i + 4]) for i in range(nd.value)]
        return {"merges": merges, "early_stop": bool(es.value), "stalled": bool(st.value),
                "need_list": int(nl.value), "need_win": int(nwn.value)}

    def symbols(self):
        n = C.c_uint64()
        self._lib.check(self.lib.gbpe_trainer_symbols(self.t, None, 0, C.byref(n)), self.ctx, "symbols")
        out = (C.c_uint32 * max(1, n.value))()
        self._lib.check(self.lib.gbpe_trainer_symbols(self.t, out, n.value, C.byref(n)), self.ctx, "symbols")
        return np.frombuffer(out, dtype=np.uint32, count=n.value).copy()

    def stats(self):
        st = self._lib.TrainerStats()
        self.lib.gbpe_trainer_stats_get(self.t, C.byref(st))
        return st

    def close(self):
        if self.t:
            self.lib.gbpe_trainer_destroy(self.t)
            self.t = None
        if self.comm and self.owns_comm:
            self.lib.gbpe_comm_destroy(self.comm)
        self.comm = None


def state_lens(lib, ctx, t):
    """(current, previous) stream lengths of a trainer (gbpe_trainer_export_state, no copy)."""
    from . import _lib
    n, npv = C.c_uint64(), C.c_uint64()
    _lib.check(lib.gbpe_trainer_export_state(t, None, 0, C.byref(n), None, 0, C.byref(npv), 0), ctx, "export_state")
    return int(n.value), int(npv.value)


def export_state(lib, ctx, t):
    """(current, previous) stream of a trainer as host u32 arrays."""
    from . import _lib
    n, npv = state_lens(lib, ctx, t)
    cur = np.zeros(max(1, n), np.uint32)
    prev = np.zeros(max(1, npv), np.uint32)
    a, b = C.c_uint64(), C.c_uint64()
    _lib.check(lib.gbpe_trainer_export_state(t, cur.ctypes.data_as(C.c_void_p), n, C.byref(a),
                                             prev.ctypes.data_as(C.c_void_p), npv, C.byref(b), 0),
               ctx, "export_state")
    return cur[:n], prev[:npv]


def export_state_device(lib, ctx, t, cur_ptr: int, prev_ptr: int, cap_cur: int, cap_prev: int):
    """The same into device buffers (HBM to HBM)."""
    from . import _lib
    a, b = C.c_uint64(), C.c_uint64()
    _lib.check(lib.gbpe_trainer_export_state(t, C.c_void_p(cur_ptr), cap_cur, C.byref(a), C.c_void_p(prev_ptr),
                                             cap_prev, C.byref(b), 1), ctx, "export_state")
    return int(a.value), int(b.value)


class GpuSingleBackend:
    """The consolidated run: one device's trainer continuing from a gathered
    state (gbpe_trainer_create_from_state) with the single-GPU policy."""

    def __init__(self, lib, ctx, cur, prev, target_vocab: int, next_id: int, exact: bool = False, flags: int = 0,
                 table_log2: int = 0, batch: int = BATCH_SIZE):
        from . import _lib
        self.lib, self.ctx, self._lib = lib, ctx, _lib
        flags |= _lib.GBPE_TRAIN_EXACT_COMPACTION if exact else 0
        self.opts = _lib.TrainOpts(target_vocab_size=target_vocab, vocab_size=next_id, next_token_id=next_id,
                                   batch_size=batch, flags=flags, table_log2=table_log2)
        t = C.c_void_p()
        if hasattr(cur, "data_ptr"):   # torch tensors (int32 / uint32 view) already in HBM
            cur, prev = cur.contiguous(), prev.contiguous()
            assert cur.is_cuda and prev.is_cuda and cur.element_size() == 4 and prev.element_size() == 4
            args = (C.c_void_p(cur.data_ptr()), cur.numel(), C.c_void_p(prev.data_ptr()), prev.numel(), 1)
        else:
            cur = np.ascontiguousarray(cur, dtype=np.uint32)
            prev = np.ascontiguousarray(prev, dtype=np.uint32)
            args = (cur.ctypes.data_as(C.c_void_p), cur.shape[0], prev.ctypes.data_as(C.c_void_p), prev.shape[0], 0)
        _lib.check(lib.gbpe_trainer_create_from_state(ctx, *args, C.byref(self.opts), C.byref(t)), ctx,
                   "create_from_state")
        self.t = t
        self.batch = batch
        self._out = (C.c_uint32 * (4 * batch))()

    def step(self, max_merges):
        nd, es = C.c_uint32(), C.c_uint32()
        self._lib.check(self.lib.gbpe_trainer_step(self.t, min(max_merges, self.batch), self._out, C.byref(nd),
                                                   C.byref(es)), self.ctx, "single step")
        return [list(self._out[4 * i: 4 * i + 4]) for i in range(nd.value)], bool(es.value)

    def symbols(self):
        n = C.c_uint64()
        self._lib.check(self.lib.gbpe_trainer_symbols(self.t, None, 0, C.byref(n)), self.ctx, "symbols")
        out = np.zeros(max(1, n.value), np.uint32)
        self._lib.check(self.lib.gbpe_trainer_symbols(self.t, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value,
                                                      C.byref(n)), self.ctx, "symbols")
        return out[: n.value]

    def stats(self):
        st = self._lib.TrainerStats()
        self.lib.gbpe_trainer_stats_get(self.t, C.byref(st))
        return st

    def close(self):
        if self.t:
            self.lib.gbpe_trainer_destroy(self.t)
            self.t = None
