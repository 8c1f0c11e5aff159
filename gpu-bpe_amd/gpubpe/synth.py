"""Seeded synthetic corpora for the benchmark configurations.

There is no network and no dataset on the GPU box, so every bench input is
generated here from a fixed seed with numpy's PCG64 (deterministic across
machines for a given numpy major version).  Corpora are word streams:

* ``english``  — Zipf(s=1.1) over a 50,000-word synthetic English-like
  lexicon (SURVEY §8(d) says 5,000; with 5k forms a 100 MiB corpus is fully
  merged after ~24K merges and a 32K-vocab run stops early), single spaces, a newline every 8-16 words, ',' / '.' with p=0.05,
  optionally 0.5 % 3-byte punctuation (’ “ ” —) — configs C1, C2.
* ``multilingual`` — per-paragraph script mix: Latin/English 50 %, Turkish
  15 %, Cyrillic 15 %, CJK 10 %, Arabic 5 %, emoji 5 % — configs C3, C4.
* ``code`` — code-like ASCII (indent runs, identifiers, numbers, operators)
  — config C5.

Generation is vectorised (piece table + gather) so 1 GiB takes seconds.
"""
from __future__ import annotations

import numpy as np

_EN_LETTERS = "etaoinshrdlcumwfgypbvkjxqz"
_EN_FREQ = np.array([12.7, 9.1, 8.2, 7.5, 7.0, 6.7, 6.3, 6.1, 6.0, 4.3, 4.0, 2.8, 2.8, 2.4,
                     2.4, 2.2, 2.0, 2.0, 1.9, 1.5, 1.0, 0.8, 0.15, 0.15, 0.1, 0.07])
_EN_FREQ = _EN_FREQ / _EN_FREQ.sum()


def _zipf_p(n: int, s: float = 1.1) -> np.ndarray:
    p = 1.0 / np.arange(1, n + 1, dtype=np.float64) ** s
    return p / p.sum()


def _alpha_lexicon(rng, alphabet: list[str], n: int, probs=None, min_len=1, mean_extra=4.0,
                   max_len=14, cap_frac=0.0) -> list[bytes]:
    words, seen = [], set()
    while len(words) < n:
        L = int(min(max_len, min_len + rng.poisson(mean_extra)))
        idx = rng.choice(len(alphabet), size=L, p=probs)
        w = "".join(alphabet[i] for i in idx)
        if cap_frac and rng.random() < cap_frac:
            w = w[:1].upper() + w[1:]
        if w in seen:
            continue
        seen.add(w)
        words.append(w.encode("utf-8"))
    # shorter words tend to get the higher Zipf ranks, as in natural text
    noise = rng.normal(0.0, 1.5, size=len(words))
    order = np.argsort(np.array([len(w.decode("utf-8")) for w in words]) + noise, kind="stable")
    return [words[i] for i in order]


def english_lexicon(seed: int = 1000, n: int = 50000) -> list[bytes]:
    rng = np.random.Generator(np.random.PCG64(seed))
    return _alpha_lexicon(rng, list(_EN_LETTERS), n, probs=_EN_FREQ, min_len=1, mean_extra=4.5, cap_frac=0.04)


def _script_lexicons(seed: int = 2000, n: int = 5000) -> dict:
    rng = np.random.Generator(np.random.PCG64(seed))
    tr = list("abcçdefgğhıijklmnoöprsştuüvyz")
    cyr = [chr(c) for c in range(0x430, 0x450)]
    ara = [chr(c) for c in range(0x627, 0x64B)]
    cjk = [chr(c) for c in rng.choice(np.arange(0x4E00, 0x9FA5), size=3000, replace=False)]
    emo = [chr(c) for c in range(0x1F600, 0x1F650)] + [chr(c) for c in range(0x1F300, 0x1F340)]
    return {
        "latin": english_lexicon(seed + 1, n),
        "turkish": _alpha_lexicon(rng, tr, n, cap_frac=0.04),
        "cyrillic": _alpha_lexicon(rng, cyr, n, cap_frac=0.04),
        "cjk": _alpha_lexicon(rng, cjk, n, min_len=1, mean_extra=1.0, max_len=4),
        "arabic": _alpha_lexicon(rng, ara, n, min_len=2, mean_extra=3.0),
        "emoji": _alpha_lexicon(rng, emo, min(n, 2000), min_len=1, mean_extra=0.3, max_len=3),
    }


def _assemble(pieces: list[bytes], ids: np.ndarray) -> np.ndarray:
    """Concatenate pieces[ids] into one uint8 array (vectorised gather)."""
    lens = np.array([len(p) for p in pieces], dtype=np.int64)
    flat = np.frombuffer(b"".join(pieces), dtype=np.uint8)
    starts = np.zeros(len(pieces), dtype=np.int64)
    starts[1:] = np.cumsum(lens)[:-1]
    L = lens[ids]
    total = int(L.sum())
    out_off = np.zeros(len(ids), dtype=np.int64)
    out_off[1:] = np.cumsum(L)[:-1]
    src = np.repeat(starts[ids] - out_off, L) + np.arange(total, dtype=np.int64)
    return flat[src]


def _word_stream(rng, lex: list[bytes], n_bytes: int, fancy_punct: float, space_sep: bool = True) -> np.ndarray:
    """Words (Zipf 1.1) + separators until ``n_bytes`` are produced."""
    V = len(lex)
    p = _zipf_p(V)
    sp = b" " if space_sep else b""
    seps = [sp, b"," + sp, b"." + sp, b"\n", b",\n", b".\n",
            "’".encode() + sp, " “".encode(), "”".encode() + sp, " —".encode() + sp]
    pieces = list(lex) + seps
    avg = float(np.dot(p, [len(w) for w in lex])) + 1.0
    out, have = [], 0
    while have < n_bytes:
        W = int(min(8_000_000, max(1024, (n_bytes - have) / avg * 1.05)))
        words = rng.choice(V, size=W, p=p)
        # newline after every 8-16 words
        gaps = rng.integers(8, 17, size=W // 8 + 2)
        nl_pos = np.cumsum(gaps)
        nl_pos = nl_pos[nl_pos < W]
        is_nl = np.zeros(W, dtype=bool)
        is_nl[nl_pos] = True
        u = rng.random(W)
        punct = np.where(u < 0.05, 1, np.where(u < 0.10, 2, 0))          # ',' / '.' p = 0.05 each
        sep = np.where(is_nl, 3 + punct, punct)
        if fancy_punct > 0:
            f = rng.random(W) < fancy_punct
            sep = np.where(f & ~is_nl, 6 + rng.integers(0, 4, size=W), sep)
        ids = np.empty(2 * W, dtype=np.int64)
        ids[0::2] = words
        ids[1::2] = V + sep
        chunk = _assemble(pieces, ids)
        out.append(chunk)
        have += chunk.shape[0]
    return np.concatenate(out)[:n_bytes]


def english(n_bytes: int, seed: int = 1, fancy_punct: float = 0.0) -> bytes:
    """C1 (fancy_punct=0) / C2 (fancy_punct=0.005) English-like text."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return _word_stream(rng, english_lexicon(), n_bytes, fancy_punct).tobytes()


def multilingual(n_bytes: int, seed: int = 3) -> bytes:
    """C3/C4: per-paragraph script mix: each paragraph
    (8-16 words, newline-terminated) is drawn from one script."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lex = _script_lexicons()
    names = ["latin", "turkish", "cyrillic", "cjk", "arabic", "emoji"]
    w = np.array([0.50, 0.15, 0.15, 0.10, 0.05, 0.05])
    pieces, off, size = [], [], []
    for name in names:
        off.append(len(pieces)); size.append(len(lex[name])); pieces += lex[name]
    sep0 = len(pieces)
    #            0     1      2      3     4      5      6    7    8
    pieces += [b" ", b", ", b". ", b"\n", b",\n", b".\n", b"", b",", b"."]
    off, size = np.array(off), np.array(size)
    avg = 7.0
    cdf = np.cumsum(_zipf_p(5000))
    out, have = [], 0
    while have < n_bytes:
        P = int(min(1_000_000, max(64, (n_bytes - have) / (12 * avg) * 1.1)))
        script = rng.choice(len(names), size=P, p=w)
        nw = rng.integers(8, 17, size=P)
        W = int(nw.sum())
        ws = np.repeat(script, nw)
        rank = np.minimum(np.searchsorted(cdf, rng.random(W)), 4999) % size[ws]
        words = off[ws] + rank
        last = np.zeros(W, dtype=bool)
        last[np.cumsum(nw) - 1] = True
        u = rng.random(W)
        punct = np.where(u < 0.05, 1, np.where(u < 0.10, 2, 0))
        cjk = ws == names.index("cjk")
        sep = np.where(last, 3 + punct, np.where(cjk, np.where(punct == 0, 6, 6 + punct), punct))
        ids = np.empty(2 * W, dtype=np.int64)
        ids[0::2] = words
        ids[1::2] = sep0 + sep
        chunk = _assemble(pieces, ids)
        out.append(chunk)
        have += chunk.shape[0]
    return np.concatenate(out)[:n_bytes].tobytes()


def code(n_bytes: int, seed: int = 6) -> bytes:
    """C5: code-like ASCII — indentation runs of 0-16 spaces, identifiers,
    1-10 digit numbers, operator/punctuation runs, comments with 's etc."""
    rng = np.random.Generator(np.random.PCG64(seed))
    idents = _alpha_lexicon(rng, list("abcdefghijklmnopqrstuvwxyz_") + list("ABCDEFGHIJKLMNOPQRSTUVWXYZ"),
                            3000, min_len=1, mean_extra=5.0, max_len=20)
    kw = [b"if", b"else", b"for", b"while", b"return", b"def", b"class", b"int", b"const",
          b"let", b"var", b"import", b"from", b"self", b"None", b"true", b"false", b"new"]
    ops = [b"(", b")", b"{", b"}", b"[", b"]", b";", b",", b".", b":", b"=", b"==", b"+=", b"->",
           b"+", b"-", b"*", b"/", b"<", b">", b"&&", b"||", b"!", b"\"", b"'", b"#", b"//"]
    nums = [str(int(x)).encode() for x in rng.integers(0, 10 ** rng.integers(1, 11, size=2000), dtype=np.int64)]
    comment_words = [w for w in english_lexicon()[:2000]] + [b"it's", b"don't", b"we're", b"I'll", b"you've"]
    indents = [b"\n" + b" " * k for k in range(0, 17)]
    pieces = idents + kw + ops + nums + comment_words + indents + [b" "]
    o_id, o_kw, o_op = 0, len(idents), len(idents) + len(kw)
    o_num = o_op + len(ops)
    o_cw = o_num + len(nums)
    o_ind = o_cw + len(comment_words)
    sp = len(pieces) - 1
    out, have = [], 0
    pid = _zipf_p(len(idents))
    pcw = _zipf_p(len(comment_words))
    while have < n_bytes:
        T = 2_000_000
        kind = rng.choice(6, size=T, p=[0.38, 0.10, 0.30, 0.07, 0.07, 0.08])
        ids = np.empty(T, dtype=np.int64)
        m = kind == 0; ids[m] = o_id + rng.choice(len(idents), size=int(m.sum()), p=pid)
        m = kind == 1; ids[m] = o_kw + rng.integers(0, len(kw), size=int(m.sum()))
        m = kind == 2; ids[m] = o_op + rng.integers(0, len(ops), size=int(m.sum()))
        m = kind == 3; ids[m] = o_num + rng.integers(0, len(nums), size=int(m.sum()))
        m = kind == 4; ids[m] = o_cw + rng.choice(len(comment_words), size=int(m.sum()), p=pcw)
        m = kind == 5; ids[m] = o_ind + rng.integers(0, 17, size=int(m.sum()))
        # a space after identifiers/keywords/numbers half the time
        need_sp = ((kind <= 1) | (kind == 3) | (kind == 4)) & (rng.random(T) < 0.5)
        full = np.empty(T + int(need_sp.sum()), dtype=np.int64)
        pos = np.arange(T) + np.concatenate([[0], np.cumsum(need_sp)[:-1]])
        full[pos] = ids
        full[pos[need_sp] + 1] = sp
        chunk = _assemble(pieces, full)
        out.append(chunk)
        have += chunk.shape[0]
    return np.concatenate(out)[:n_bytes].tobytes()


def shard_at_word_starts(data: bytes, world: int, word_starts: np.ndarray) -> list[tuple[int, int]]:
    """Split [0, n) into ``world`` contiguous ranges cut at word-start
    positions: pairs never cross a word start."""
    n = len(data)
    cuts = [0]
    ws = np.flatnonzero(word_starts)
    for r in range(1, world):
        target = n * r // world
        k = int(np.searchsorted(ws, target))
        c = int(ws[k]) if k < ws.shape[0] else n
        cuts.append(max(c, cuts[-1]))
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]
