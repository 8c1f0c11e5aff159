"""One input encoded by R ranks: chunk-aligned slices, an
exclusive scan of the R token totals, a gather.

The reference already cuts its input into chunk-aligned pieces per dispatch
(tokenizer.js:181-203) and every chunk is an independent greedy walk
(tokenize.wgsl:88-175), so slices that start at multiples of the chunk size
encode to exactly the tokens of one pass.  Rank r encodes slice r on its own GPU
with no data-path collective; one all-gather of R integers gives each slice's
output offset (the scan that trie_prefix_sum does per chunk, tokenize.wgsl:
199-208, lifted to slices); the tokens are then gathered where they are needed.

``encode`` is any callable bytes -> uint32 tokens (TrieTokenizer.encode_bytes on
the GPU; the CPU oracle in the gloo tests).  ``dist`` is torch.distributed,
initialised; ``device`` is where collective tensors live ("cuda" for RCCL,
"cpu" for gloo).
"""
from __future__ import annotations

import numpy as np


def slice_bounds(n: int, chunk: int, world: int) -> list[tuple[int, int]]:
    """Balanced [start, end) byte ranges, every start a multiple of `chunk`."""
    nch = -(-n // chunk) if n else 0
    out, c = [], 0
    for r in range(world):
        c1 = nch * (r + 1) // world
        out.append((min(c * chunk, n), min(c1 * chunk, n)))
        c = c1
    return out


def _all_gather_counts(dist, local: int, device: str) -> list[int]:
    import torch
    t = torch.tensor([local], dtype=torch.int64, device=device)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def encode_split(encode, data: bytes, chunk: int, dist, device: str = "cpu", gather_to: int | None = 0):
    """Encode `data` across the ranks of `dist`.  Returns (tokens, offsets,
    counts): tokens is the full uint32 token array on `gather_to` (on every rank
    when gather_to is None, None elsewhere); offsets[r] / counts[r] place slice
    r's tokens in it."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    s, e = slice_bounds(len(data), chunk, world)[rank]
    local = np.ascontiguousarray(encode(data[s:e]) if e > s else np.zeros(0, np.uint32), dtype=np.uint32)
    counts = _all_gather_counts(dist, int(local.shape[0]), device)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64).tolist()
    total = int(sum(counts))
    cap = max(counts) if counts else 0
    # variable-size gather as one padded all-gather (gloo and RCCL alike); int32
    # carries the u32 ids bit for bit
    buf = torch.zeros(cap, dtype=torch.int32, device=device)
    if local.shape[0]:
        buf[: local.shape[0]] = torch.from_numpy(local.view(np.int32)).to(device)
    if gather_to is None or world == 1:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
    else:
        parts = [torch.empty_like(buf) for _ in range(world)] if rank == gather_to else None
        if device == "cpu":
            dist.gather(buf, parts, dst=gather_to)
        else:   # RCCL: all-gather (gather is not offered by every build); the other ranks drop theirs
            tmp = [torch.empty_like(buf) for _ in range(world)]
            dist.all_gather(tmp, buf)
            parts = tmp if rank == gather_to else None
    if parts is None:
        return None, offsets, counts
    out = np.empty(total, dtype=np.uint32)
    for r in range(world):
        out[offsets[r]: offsets[r] + counts[r]] = parts[r][: counts[r]].cpu().numpy().view(np.uint32)
    return out, offsets, counts
