"""CPU oracle for the gpu-bpe hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``gpu-bpe_amd/``) never routes through it and fails loudly
when the HIP library is missing.

It restates, in numpy / plain Python, the behaviour of the reference
toprakdeviren/gpu-bpe (read-only at /root/reference) for the two hot paths:

* BPE training merge loop — ``src/bpe/train.wgsl`` driven by
  ``src/bpe/training-pipeline.js`` and ``src/bpe/trainer.js``;
* chunked greedy trie encode — ``src/bpe/tokenizer/tokenize.wgsl`` driven by
  ``src/bpe/tokenizer/tokenizer.js``, plus the trie compiler
  ``src/bpe/tokenizer/trie.js`` and the vocabulary ``src/bpe/vocab.js``.

Pinning: the CPU-side reference modules (vocab.js,
trie.js, tokenizer-manager.js) are executed under Node 12 in the dev
container by ``oracle/ref_js/run_ref_modules.mjs`` and their outputs are the
golden fixtures in ``tests/golden/``.  The WGSL kernels cannot execute here
(no WebGPU runtime); their restatement below is pinned by the hand-derived
known answers in ``tests/golden/known_answers.json`` — parity for the kernel
semantics is therefore *partially pinned*.

Two reference behaviours that the restatement reproduces on purpose:

1. **Snapshot merge** (train.wgsl:476 "Read ALL inputs BEFORE any writes").
   The reference writes ``symbols[id]`` in place while neighbours read it
   (train.wgsl:477-487); we take the race-free snapshot semantics.
2. **Compaction tail drop** (train.wgsl:605-607 + 698/727).  The scan kernel
   stores the NEW symbol count into ``state.symbol_count`` and the following
   ``bpe_finalize_compact_b`` bounds its scatter with that same field, so
   valid symbols whose OLD index is >= the new count are never scattered:
   the last ``m`` slots of the compacted stream keep whatever the ping-pong
   destination buffer held (zeros from WebGPU's zero-initialised buffer on
   the first merge, then the in-place-rewritten stream from two merges
   before).  ``compaction="exact"`` gives the intended (bug-free) result.
"""
from __future__ import annotations

import json
import numpy as np

WORD_START_BIT = 0x10000          # train.wgsl:36
TOKEN_MASK = 0xFFFF               # train.wgsl:37
INVALID_TOKEN = 0xFFFFFFFF        # engine.js:12 / tokenize.wgsl:20
TABLE_SIZE = 1 << 21              # engine.js:11
BATCH_SIZE = 128                  # training-pipeline.js:13
DEFAULT_CHUNK_SIZE = 512          # tokenizer.js:17
TRIE_MAGIC = 0x54524945           # trie.js:20
TRIE_VERSION = 3                  # trie.js:21
TRIE_HEADER_SIZE = 28             # trie.js:23
UTF8_REPLACEMENT = [0xEF, 0xBF, 0xBD]   # tokenizer.js:18


# ─────────────────────────────── word boundaries ──────────────────────────────

def char_class_array(tok: np.ndarray) -> np.ndarray:
    """Byte class, train.wgsl:111-127: \\n→4, space→2, digit→1, letter/≥0x80→0, else 3."""
    tok = tok.astype(np.uint32)
    cls = np.full(tok.shape, 3, dtype=np.uint8)
    letter = (tok >= 0x80) | ((tok >= 0x61) & (tok <= 0x7A)) | ((tok >= 0x41) & (tok <= 0x5A))
    cls[letter] = 0
    cls[(tok >= 0x30) & (tok <= 0x39)] = 1
    cls[tok == 0x20] = 2
    cls[tok == 0x0A] = 4
    return cls


def heuristic_word_starts(data: np.ndarray) -> np.ndarray:
    """Word-start mask of ``bpe_word_boundary`` (train.wgsl:144-186), bool[n]."""
    n = data.shape[0]
    ws = np.zeros(n, dtype=bool)
    if n == 0:
        return ws
    cls = char_class_array(data)
    prev, cur = cls[:-1], cls[1:]
    b = prev != cur                                            # :165
    b &= ~((prev == 2) & ((cur == 0) | (cur == 1)))            # :168-170
    b |= (cur == 2) & (prev != 2)                              # :173-175
    b |= (prev == 4) | (cur == 4)                              # :178-180
    ws[0] = True                                               # :156-159
    ws[1:] = b
    return ws


def prepare_symbols(data: bytes | np.ndarray, word_starts=None) -> np.ndarray:
    """Byte → u32 symbol with bit16 = word start.

    External mask: trainer.js:115-121 (tagWordBoundaries).  No mask: the GPU
    heuristic (trainer.js:177-180 → train.wgsl:144-186).
    """
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data.astype(np.uint8)
    sym = arr.astype(np.uint32)
    if word_starts is not None:
        ws = np.asarray(word_starts).astype(bool)
        assert ws.shape[0] == sym.shape[0]
    else:
        ws = heuristic_word_starts(arr)
    sym[ws] |= WORD_START_BIT
    return sym


# ─────────────────────────────── training loop ────────────────────────────────

def count_pairs(s: np.ndarray):
    """Exact pair counts of one stream, train.wgsl:393-399.

    A pair (i-1, i) counts iff symbol i has no word-start bit and neither
    token is 0.  Returns (unique pids ascending, counts)."""
    if s.shape[0] < 2:
        return np.zeros(0, np.uint32), np.zeros(0, np.int64)
    tok = s & TOKEN_MASK
    m = ((s[1:] & WORD_START_BIT) == 0) & (tok[:-1] != 0) & (tok[1:] != 0)
    pids = ((tok[:-1][m] << 16) | tok[1:][m]).astype(np.uint32)
    if pids.size == 0:
        return np.zeros(0, np.uint32), np.zeros(0, np.int64)
    return np.unique(pids, return_counts=True)


def select_best(uniq: np.ndarray, counts: np.ndarray):
    """Deterministic argmax (train.wgsl:83-85): higher count, then smaller pid."""
    if uniq.size == 0:
        return 0, 0
    i = int(np.argmax(counts))          # first max → smallest pid (uniq is ascending)
    return int(counts[i]), int(uniq[i])


def merge_step(cur: np.ndarray, oth: np.ndarray, n: int, a: int, b: int, new: int,
               compaction: str = "reference") -> tuple[int, int]:
    """One merge on the ping-pong pair (cur → oth), snapshot semantics.

    Follows bpe_merge_reduce_b (train.wgsl:475-500), the block scan
    (train.wgsl:641-651) and bpe_finalize_compact_b (train.wgsl:693-730).
    Mutates ``cur`` in place (A-side rewrite, train.wgsl:482-488) and
    ``oth``.  Returns (new_n, m) where m = valid symbols dropped by the
    reference's compaction bound (0 for compaction="exact")."""
    s = cur[:n].copy()                      # snapshot: all reads before any write
    tok = s & TOKEN_MASK
    hit = np.zeros(n, dtype=bool)           # hit[i]: pair (i-1, i) == (a, b), train.wgsl:491-497
    if n >= 2:
        hit[1:] = ((s[1:] & WORD_START_BIT) == 0) & (tok[:-1] == a) & (tok[1:] == b)
    rw = np.zeros(n, dtype=bool)            # A-side rewrite, train.wgsl:482-485
    rw[:-1] = hit[1:]
    valid = ~hit
    cur[:n][rw] = np.uint32(new) | (s[rw] & WORD_START_BIT)
    new_n = int(valid.sum())
    idx = np.flatnonzero(valid)
    if compaction == "reference":
        keep = idx[idx < new_n]             # fid < state.symbol_count (already the NEW count)
        oth[:keep.shape[0]] = cur[keep]
        m = new_n - keep.shape[0]
    elif compaction == "exact":
        oth[:new_n] = cur[idx]
        m = 0
    else:
        raise ValueError(compaction)
    return new_n, m


class TrainResult(dict):
    pass


def train(data, target_vocab_size: int = 4096, word_starts=None, next_token_id: int = 256,
          vocab_size: int | None = None, compaction: str = "reference",
          keep_history: bool = False, max_merges: int | None = None) -> TrainResult:
    """Full training restatement (trainer.js:149-220, 225-335 + train.wgsl).

    Returns dict(merges=[[a, b, id, count], ...], symbols=final stream u32,
    n_history=[N_0, N_1, ...], early_stop=bool).
    ``vocab_size`` defaults to ``next_token_id`` (a fresh Vocab has size 256 =
    nextTokenId, vocab.js:92-124)."""
    sym = prepare_symbols(data, word_starts)
    n0 = sym.shape[0]
    if n0 == 0:
        raise ValueError("No symbols to train on — corpus is empty after pre-processing")
    if vocab_size is None:
        vocab_size = next_token_id
    needed = target_vocab_size - vocab_size               # trainer.js:208
    if max_merges is not None:
        needed = min(needed, max_merges)
    A = sym.copy()
    B = np.zeros(n0, dtype=np.uint32)                      # WebGPU buffers are zero-initialised
    cur, oth = A, B
    n = n0
    nxt = next_token_id
    merges, hist, tails = [], [n0], []
    early = False
    while len(merges) < needed:
        uniq, counts = count_pairs(cur[:n])
        mc, pid = select_best(uniq, counts)
        if mc < 2 or nxt > TOKEN_MASK:                     # train.wgsl:345-348
            early = True
            break
        a, b = pid >> 16, pid & 0xFFFF
        n, m = merge_step(cur, oth, n, a, b, nxt, compaction)
        merges.append([a, b, nxt, mc])
        nxt += 1
        cur, oth = oth, cur
        hist.append(n)
        tails.append(m)
    res = TrainResult(merges=merges, symbols=cur[:n].copy(), n_history=hist,
                      tail_drops=tails, early_stop=early, next_token_id=nxt)
    return res


# ─────────────────────────────── vocabulary ───────────────────────────────────

def _fmt_hex(b: int) -> str:
    return "<0x%02X>" % b


def _fmt_ascii(b: int) -> str:
    if b == 0x20:
        return "▁"
    if b == 0x0A:
        return "\\n"
    if 0x21 <= b <= 0x7E:
        return chr(b)
    return _fmt_hex(b)


def bytes_to_display_string(bs) -> str:
    """vocab.js:18-53 (UTF-8 where valid, ▁ for space, hex otherwise)."""
    parts, i, n = [], 0, len(bs)
    while i < n:
        b = bs[i]
        if b < 0x80:
            parts.append(_fmt_ascii(b)); i += 1; continue
        if b < 0xC0:
            parts.append(_fmt_hex(b)); i += 1; continue
        L = 2 if b < 0xE0 else 3 if b < 0xF0 else 4
        dec = None
        if i + L <= n and all((bs[i + j] & 0xC0) == 0x80 for j in range(1, L)):
            try:
                dec = bytes(bs[i:i + L]).decode("utf-8", errors="strict")
            except UnicodeDecodeError:
                dec = None
        if dec is not None:
            parts.append(dec); i += L
        else:
            parts.append(_fmt_hex(b)); i += 1
    return "".join(parts)


class Vocab:
    """vocab.js:92-144."""

    def __init__(self):
        self.entries = [[i] for i in range(256)]
        self.strings = [bytes_to_display_string([i]) for i in range(256)]
        self.next_token_id = 256

    @property
    def size(self):
        return len(self.entries)

    def add_merge(self, a: int, b: int) -> int:
        nid = self.next_token_id
        self.next_token_id += 1
        merged = list(self.entries[a]) + list(self.entries[b])
        self.entries.append(merged)
        self.strings.append(bytes_to_display_string(merged))
        return nid

    def export(self) -> str:
        lines = ["# GPU BPE Vocabulary (WebGPU Trainer)", f"# Total tokens: {len(self.entries)}", ""]
        for i, e in enumerate(self.entries):
            lines.append(f"{i}\t{self.strings[i]}\t[{','.join(str(x) for x in e)}]")
        return "\n".join(lines) + "\n"


def vocab_from_merges(merges) -> Vocab:
    v = Vocab()
    for m in merges:
        v.add_merge(m[0], m[1])
    return v


# ─────────────────────────────── trie (v3) ────────────────────────────────────

def compile_vocab_to_trie(vocab) -> bytes:
    """trie.js:39-98 + serializeTrie trie.js:167-206 (BFS, children sorted by
    byte, a later duplicate byte string overwrites the tokenId)."""
    root = {"c": {}, "t": INVALID_TOKEN}
    max_len = 0
    for tid, bs in enumerate(vocab):
        if not bs:
            continue
        node = root
        for byte in bs:
            node = node["c"].setdefault(byte, {"c": {}, "t": INVALID_TOKEN})
        node["t"] = tid
        max_len = max(max_len, len(bs))
    nodes, edges = [None], []
    queue, head = [root], 0
    index = {id(root): 0}
    while head < len(queue):
        tn = queue[head]; head += 1
        me = index[id(tn)]
        first = len(edges)
        kids = sorted(tn["c"].items())
        for sym, child in kids:
            ci = len(queue)
            index[id(child)] = ci
            queue.append(child)
            nodes.append(None)
            edges.append((sym, ci))
        nodes[me] = (first, len(kids), tn["t"])
    hdr = np.array([TRIE_MAGIC, TRIE_VERSION, len(nodes), len(edges), max_len, len(vocab), 0], dtype="<u4")
    nd = np.array(nodes, dtype="<u4").reshape(-1, 3) if nodes else np.zeros((0, 3), "<u4")
    ed = np.zeros((len(edges), 2), dtype="<u4")
    if edges:
        ed[:, 0] = [e[0] for e in edges]            # symbol u8 + 3 zero pad bytes
        ed[:, 1] = [e[1] for e in edges]
    return hdr.tobytes() + nd.tobytes() + ed.tobytes()


def parse_header(data: bytes) -> dict:
    """trie.js:110-128."""
    h = np.frombuffer(data[:TRIE_HEADER_SIZE], dtype="<u4")
    if int(h[0]) != TRIE_MAGIC:
        raise ValueError("Invalid trie magic: 0x%x" % int(h[0]))
    if int(h[1]) not in (2, 3):
        raise ValueError("Unsupported trie version: %d" % int(h[1]))
    return dict(version=int(h[1]), nodeCount=int(h[2]), edgeCount=int(h[3]), maxTokenLen=int(h[4]))


def parse_trie_buffers(data: bytes, header: dict):
    """trie.js:137-160, 209-249 → (nodes u32[3N], edges u32[2E])."""
    v, nc, ec = header["version"], header["nodeCount"], header["edgeCount"]
    bpn, bpe = (12, 8) if v == 3 else (8, 4)
    if len(data) < TRIE_HEADER_SIZE + nc * bpn + ec * bpe:
        raise ValueError("Truncated trie data")
    off = TRIE_HEADER_SIZE
    if v == 3:
        nodes = np.frombuffer(data[off:off + nc * 12], dtype="<u4").astype(np.uint32).copy()
        e = np.frombuffer(data[off + nc * 12: off + nc * 12 + ec * 8], dtype="<u4").reshape(-1, 2)
        edges = np.zeros((ec, 2), np.uint32)
        edges[:, 0] = e[:, 0] & 0xFF
        edges[:, 1] = e[:, 1]
        edges = edges.reshape(-1)
    else:
        raw = np.frombuffer(data[off:off + nc * 8], dtype="<u2").reshape(-1, 4)
        nodes = np.zeros((nc, 3), np.uint32)
        nodes[:, 0] = raw[:, 0]
        nodes[:, 1] = raw[:, 1]
        t = raw[:, 2].astype(np.uint32)
        t[t == 0xFFFF] = INVALID_TOKEN
        nodes[:, 2] = t
        nodes = nodes.reshape(-1)
        e = np.frombuffer(data[off + nc * 8: off + nc * 8 + ec * 4], dtype="<u2").reshape(-1, 2)
        edges = np.zeros((ec, 2), np.uint32)
        edges[:, 0] = e[:, 0] & 0xFF
        edges[:, 1] = e[:, 1]
        edges = edges.reshape(-1)
    return nodes, edges


def adaptive_chunk_size(max_token_len: int) -> int:
    """tokenizer.js:67-68."""
    return max(DEFAULT_CHUNK_SIZE, min(2048, max_token_len * 8))


# ─────────────────────────────── trie encode ──────────────────────────────────

def _find_child(edges, first, num, sym):
    """Branchless lower bound, tokenize.wgsl:69-86."""
    lo, n = 0, num
    while n > 0:
        half = n >> 1
        mid = lo + half
        if (int(edges[(first + mid) * 2]) & 0xFF) < sym:
            lo, n = mid + 1, n - half - 1
        else:
            n = half
    if lo < num and (int(edges[(first + lo) * 2]) & 0xFF) == sym:
        return int(edges[(first + lo) * 2 + 1])
    return INVALID_TOKEN


def encode_chunked(data: bytes, nodes, edges, chunk_size: int) -> np.ndarray:
    """Greedy longest match per chunk (tokenize.wgsl:88-175); tokens never
    cross a chunk; unmatched byte → its byte value.  Multi-pass slicing
    (tokenizer.js:181-203) is chunk aligned and therefore equal to this."""
    nodes = [int(x) for x in nodes]
    edges = [int(x) for x in edges]
    n = len(data)
    if n == 0:
        return np.zeros(0, np.uint32)
    # root LUT + depth-1 cache (tokenize.wgsl:96-117)
    root_fc, root_nc = nodes[0], nodes[1] & 0xFFFF
    lut = [INVALID_TOKEN] * 256
    for k in range(min(root_nc, 256)):
        lut[edges[(root_fc + k) * 2] & 0xFF] = edges[(root_fc + k) * 2 + 1]
    out = []
    for cs in range(0, n, chunk_size):
        ce = min(cs + chunk_size, n)
        pos = cs
        while pos < ce:
            cn, lmt, lmp, wp, depth = 0, INVALID_TOKEN, pos, pos, 0
            while wp < ce:
                bv = data[wp]
                if cn == 0 and depth == 0:
                    nn = lut[bv]
                else:
                    nn = _find_child(edges, nodes[cn * 3], nodes[cn * 3 + 1] & 0xFFFF, bv)
                if nn == INVALID_TOKEN:
                    break
                cn = nn; wp += 1; depth += 1
                ti = nodes[cn * 3 + 2]
                if ti != INVALID_TOKEN:
                    lmt, lmp = ti, wp
            if lmt != INVALID_TOKEN:
                out.append(lmt); pos = lmp
            else:
                out.append(data[pos]); pos += 1
    return np.array(out, dtype=np.uint32)


def decode(tokens, vocab) -> bytes:
    """tokenizer.js:344-363 (unknown ids → U+FFFD bytes)."""
    out = bytearray()
    for t in tokens:
        t = int(t)
        out.extend(vocab[t] if t < len(vocab) else UTF8_REPLACEMENT)
    return bytes(out)


def encode_merge_order(data: bytes, merges) -> list:
    """CPU merge-order encoder of the UI tab (tokenizer-manager.js:13-61)."""
    if not merges:
        return list(data)
    tokens = list(data)
    for a, b, nid in (m[:3] for m in merges):
        if len(tokens) < 2:
            break
        out, i, L = [], 0, len(tokens)
        while i < L:
            if i + 1 < L and tokens[i] == a and tokens[i + 1] == b:
                out.append(nid); i += 2
            else:
                out.append(tokens[i]); i += 1
        tokens = out
    return tokens


def dxft_bin(tokens, vocab_size: int, vocab_json: dict | None) -> bytes:
    """.bin export, export-controller.js:221-248: u32 [MAGIC, vocabSize,
    tokenCount, vocabJsonLen, tokens...] + vocab JSON bytes."""
    vb = json.dumps(vocab_json, separators=(",", ":")).encode() if vocab_json is not None else b""
    hdr = np.array([0x44584654, vocab_size, len(tokens), len(vb)], dtype="<u4")
    return hdr.tobytes() + np.asarray(tokens, dtype="<u4").tobytes() + vb


# ─────────────────────── GPT-4 rule pre-tokenizer (word starts) ─────────────────
# Restates src/wasm/pre_tokenizer.mjs (PreTokenizer.preTokenizeBytes, :459-509)
# for already-NFC UTF-8 input: utf8ToCodepoints (:517-551), classify (:128-136),
# findWordBoundaries (:226-292), byte mapping (:497-506).  Classes come from
# Python's unicodedata here; the reference uses its Decoder WASM tables
# (Unicode 17), so non-ASCII codepoints whose category changed are unpinned.

import unicodedata as _ud

PT_LETTER, PT_DIGIT, PT_WHITESPACE, PT_PUNCT, PT_SYMBOL, PT_NEWLINE, PT_OTHER = range(7)   # :34-42
_PT_NEWLINES = {0x0A, 0x0D, 0x0085, 0x2028, 0x2029}                                        # :44
_PT_WHITE_SPACE = set(range(0x09, 0x0E)) | {0x20, 0x85, 0xA0, 0x1680} | set(range(0x2000, 0x200B)) | \
    {0x2028, 0x2029, 0x202F, 0x205F, 0x3000}                                               # PropList White_Space
_PT_SINGLE = {0x73, 0x53, 0x74, 0x54, 0x6D, 0x4D, 0x64, 0x44}                              # :56-61
_PT_TWO = [(0x72, 0x52, 0x65, 0x45), (0x76, 0x56, 0x65, 0x45), (0x6C, 0x4C, 0x6C, 0x4C)]    # :68-72
_PT_APOS = {0x27, 0x2019}                                                                  # :75


def pt_classify(cp: int) -> int:
    """classify(), pre_tokenizer.mjs:128-136 (decoder predicates as general categories)."""
    if cp in _PT_NEWLINES:
        return PT_NEWLINE
    try:
        cat = _ud.category(chr(cp))
    except ValueError:
        return PT_OTHER
    if cat[0] in "LM":
        return PT_LETTER
    if cat[0] == "N":
        return PT_DIGIT
    if cp in _PT_WHITE_SPACE:
        return PT_WHITESPACE
    if cat[0] == "P":
        return PT_PUNCT
    if cat[0] == "S":
        return PT_SYMBOL
    return PT_OTHER


def utf8_to_codepoints(b: bytes):
    """utf8ToCodepoints, pre_tokenizer.mjs:517-551: the lead byte picks the size;
    bytes past the end read as 0 (JS `undefined & 0x3F`).  Returns (cps, sizes)."""
    cps, sizes = [], []
    i, n = 0, len(b)
    at = lambda k: b[k] if k < n else 0
    while i < n:
        c = b[i]
        if c < 0x80:
            cp, sz = c, 1
        elif (c & 0xE0) == 0xC0:
            cp, sz = ((c & 0x1F) << 6) | (at(i + 1) & 0x3F), 2
        elif (c & 0xF0) == 0xE0:
            cp, sz = ((c & 0x0F) << 12) | ((at(i + 1) & 0x3F) << 6) | (at(i + 2) & 0x3F), 3
        else:
            cp, sz = (((c & 0x07) << 18) | ((at(i + 1) & 0x3F) << 12) | ((at(i + 2) & 0x3F) << 6) |
                      (at(i + 3) & 0x3F)), 4
        cps.append(cp)
        sizes.append(sz)
        i += sz
    return cps, sizes


def _utf8_len(cp: int) -> int:
    """utf8ByteLength, pre_tokenizer.mjs:301-306."""
    return 1 if cp <= 0x7F else 2 if cp <= 0x7FF else 3 if cp <= 0xFFFF else 4


def _match_contraction(cps, cls, i):
    """matchContraction, pre_tokenizer.mjs:85-114."""
    n = len(cps)
    if i + 1 >= n:
        return 0
    nxt = cps[i + 1]
    after_non_letter = i + 2 >= n or cls[i + 2] != PT_LETTER
    if nxt in _PT_SINGLE and after_non_letter:
        return 2
    if i + 2 < n:
        nn = cps[i + 2]
        after_two = i + 3 >= n or cls[i + 3] != PT_LETTER
        for lo1, hi1, lo2, hi2 in _PT_TWO:
            if nxt in (lo1, hi1) and nn in (lo2, hi2) and after_two:
                return 3
    return 0


def _class_transition(prev, curr):
    """isClassTransitionBoundary, pre_tokenizer.mjs:185-200."""
    ps = lambda c: c in (PT_PUNCT, PT_SYMBOL)
    return ((prev == PT_LETTER and curr == PT_DIGIT) or (prev == PT_DIGIT and curr == PT_LETTER) or
            (prev == PT_LETTER and ps(curr)) or (ps(prev) and curr == PT_LETTER) or
            (ps(prev) and curr == PT_DIGIT) or (prev == PT_DIGIT and ps(curr)))


def gpt4_word_starts(data: bytes) -> np.ndarray:
    """Byte-level word-start mask of PreTokenizer.preTokenizeBytes for NFC input
    (findWordBoundaries, pre_tokenizer.mjs:226-292; byte mapping :497-506)."""
    b = bytes(data)
    out = np.zeros(len(b), dtype=np.uint8)
    if not b:
        return out
    cps, _ = utf8_to_codepoints(b)
    cls = [pt_classify(c) for c in cps]
    n = len(cps)
    starts = [0] * n
    starts[0] = 1
    i = 1
    while i < n:
        prev, curr = cls[i - 1], cls[i]
        if curr == PT_NEWLINE or prev == PT_NEWLINE:
            starts[i] = 1
            i += 1
            continue
        if curr == PT_WHITESPACE:
            if prev != PT_WHITESPACE:
                starts[i] = 1
            i += 1
            continue
        if prev == PT_WHITESPACE:
            i += 1
            continue
        if prev == PT_LETTER and cps[i] in _PT_APOS:
            k = _match_contraction(cps, cls, i)
            if k > 0:
                i += k
                continue
        if _class_transition(prev, curr):
            starts[i] = 1
            i += 1
            continue
        if curr == PT_DIGIT and prev == PT_DIGIT:
            rs = i - 1
            while rs > 0 and cls[rs - 1] == PT_DIGIT:
                rs -= 1
            if (i - rs) % 3 == 0:
                starts[i] = 1
            i += 1
            continue
        i += 1
    pos = 0                                   # byte mapping by the codepoint's own length (:497-506)
    for k in range(n):
        if starts[k] and pos < len(b):
            out[pos] = 1
        pos += _utf8_len(cps[k])
    return out
