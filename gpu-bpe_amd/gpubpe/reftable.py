"""Where the reference's pair table would have dropped counts.

The reference recounts every pair of the stream each merge into a fixed
2^21-slot open-addressing table (engine.js:11) with triangular probing and gives
up after 128 probes, silently dropping that pair's count for the merge
(train.wgsl:415-430; the per-workgroup 1024-slot LDS stage, train.wgsl:393-411,
holds at most 256 distinct pairs and never fills).  This engine's table is
exact and grows, so on corpora with more distinct pairs the reference's merge
list is no longer the exact one; these helpers say where that starts.

``simulate_drops`` inserts a set of distinct pair ids into a model of the
reference table: all keys probe in lock step (one round per probe index), an
empty slot goes to the first key that wants it (atomicCompareExchangeWeak
succeeds for one workgroup), the others continue — the order the reference's
parallel flush would see is not defined, so this is an estimate, not a replay.
"""
from __future__ import annotations

import numpy as np

REF_TABLE_SIZE = 1 << 21   # engine.js:11 TABLE_SIZE
REF_MAX_PROBE = 128        # train.wgsl:33 MAX_PROBE


def pair_hash(pid: np.ndarray) -> np.ndarray:
    """Murmur3 fmix32 (train.wgsl:61-67), vectorised over uint32."""
    x = pid.astype(np.uint32)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint32(16))) * np.uint32(0x7FEB352D)
        x = (x ^ (x >> np.uint32(15))) * np.uint32(0x846CA68B)
    return x ^ (x >> np.uint32(16))


def simulate_drops(pids, table_size: int = REF_TABLE_SIZE, max_probe: int = REF_MAX_PROBE, seed: int = 0) -> int:
    """Distinct pairs of ``pids`` the reference table would fail to place."""
    keys = np.unique(np.asarray(pids, dtype=np.uint32))
    keys = keys[keys != 0]
    if keys.size == 0:
        return 0
    keys = np.random.default_rng(seed).permutation(keys)   # insertion order: undefined in the reference
    mask = np.uint32(table_size - 1)
    h = pair_hash(keys)
    occupied = np.zeros(table_size, dtype=bool)
    pending = np.arange(keys.size)
    for p in range(max_probe):
        if pending.size == 0:
            break
        idx = (h[pending] + np.uint32((p * (p + 1)) // 2)) & mask
        free = ~occupied[idx]
        cand, cidx = pending[free], idx[free]
        # one winner per empty slot (the first in order); the rest probe on
        _, first = np.unique(cidx, return_index=True)
        occupied[cidx[first]] = True
        won = np.zeros(pending.size, dtype=bool)
        won[np.flatnonzero(free)[first]] = True
        pending = pending[~won]
        del cand
    return int(pending.size)


def report(max_live_pairs: int, final_pids=None) -> dict:
    """The per-leg record: the largest live pair set against the reference
    table, and (given the final live pair ids) the simulated drops there."""
    out = {"reference_table_slots": REF_TABLE_SIZE, "max_live_pairs": int(max_live_pairs),
           "max_load_vs_reference": round(max_live_pairs / REF_TABLE_SIZE, 4),
           "exceeds_reference_table": bool(max_live_pairs > REF_TABLE_SIZE)}
    if final_pids is not None:
        n = int(np.unique(np.asarray(final_pids, dtype=np.uint32)).size)
        out["final_live_pairs"] = n
        out["final_simulated_reference_drops"] = simulate_drops(final_pids)
    out["reference_exact"] = not out["exceeds_reference_table"] and out.get("final_simulated_reference_drops", 0) == 0
    return out
