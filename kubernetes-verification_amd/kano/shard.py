"""Row partition of the reachability matrix across ranks (one process per
GPU) and the exchange step of the column checks.

Rows of M (source pods) are independent: M[i] = OR_{p in S(i)} allow_p
(kano_py/kano/model.py:158-160), so rank r builds rows [row_range(n, W, r)]
with no communication.  The column checks are existentials / universals over
rows, so they combine over shards:

  all_isolated[j]    = NOT OR_r colOR_r[j]          (algorithm.py:12-17)
  all_reachable[j]   = NOT OR_r colNAND_r[j]        (algorithm.py:4-9)
  user_crosscheck[j] = OR_r cross_r[j]              (algorithm.py:27-42)

RCCL has no bitwise reduction.  The bench's step (kano_verify_shard /
kano_verify_combine) gathers every rank's three bit vectors as words,
[or | cross | nand] (3 W u64 = n*3/8 bytes per rank), with one all-gather over
xGMI and ORs them on the device; ``combine_words`` is the host statement of
that combine.  The older byte form (``pack_flags``: one byte per column, one
MAX all-reduce, MAX of 0/1 bytes = OR) stays for kano_col_flags_dev.
system_isolation reads one row from the rank that owns it; policy_shadow's
output is ordered by container, so each rank emits its own rows' pairs and
rank order is the global order.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np


def row_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    return rank * n // world, (rank + 1) * n // world


def owner_of_row(n: int, world: int, i: int) -> int:
    for r in range(world):
        a, b = row_range(n, world, r)
        if a <= i < b:
            return r
    raise IndexError(i)


def pack_flags(col_or: np.ndarray, cross: np.ndarray, col_nand: np.ndarray, n: int) -> np.ndarray:
    """Three LSB-first word vectors -> [or | cross | nand] bytes (host side of
    kano_col_flags_dev / kano_crosscheck_dev)."""
    out = np.empty(3 * n, np.uint8)
    for k, w in enumerate((col_or, cross, col_nand)):
        b = np.unpackbits(np.ascontiguousarray(w, dtype="<u8").view(np.uint8),
                          bitorder="little")[:n]
        out[k * n:(k + 1) * n] = b
    return out


def decode_flags(flags: np.ndarray, n: int) -> Dict[str, np.ndarray]:
    """Combined [or | cross | nand] bytes -> the three check results."""
    f = np.asarray(flags)
    return {
        "all_isolated": np.flatnonzero(f[:n] == 0),
        "user_crosscheck": np.flatnonzero(f[n:2 * n]),
        "all_reachable": np.flatnonzero(f[2 * n:3 * n] == 0),
    }


def combine_words(gathered: np.ndarray, n: int) -> Dict[str, np.ndarray]:
    """Gathered [rank][or | cross | nand][W] u64 words -> the three check
    results (host statement of k_combine_cols)."""
    W = (n + 63) // 64
    g = np.asarray(gathered, dtype=np.uint64).reshape(-1, 3, W)
    o, c, na = (np.bitwise_or.reduce(g[:, k, :], axis=0) for k in range(3))

    def bits(w):
        return np.unpackbits(np.ascontiguousarray(w, dtype="<u8").view(np.uint8),
                             bitorder="little")[:n].astype(bool)
    return {
        "all_isolated": np.flatnonzero(~bits(o)),
        "user_crosscheck": np.flatnonzero(bits(c)),
        "all_reachable": np.flatnonzero(~bits(na)),
    }
