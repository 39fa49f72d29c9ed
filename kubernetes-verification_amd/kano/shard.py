"""Row partition of the reachability matrix across ranks (one process per
GPU) and the exchange step of the column checks.

Rows of M (source pods) are independent: M[i] = OR_{p in S(i)} allow_p
(kano_py/kano/model.py:158-160), so rank r builds rows [row_range(n, W, r)]
with no communication.  The column checks are existentials / universals over
rows, so they combine over shards:

  all_isolated[j]    = NOT OR_r colOR_r[j]          (algorithm.py:12-17)
  all_reachable[j]   = NOT OR_r colNAND_r[j]        (algorithm.py:4-9)
  user_crosscheck[j] = OR_r cross_r[j]              (algorithm.py:27-42)

RCCL has no bitwise reduction, so each rank unpacks its three bit vectors to
one byte per column, [or | cross | nand] (3n bytes), and one MAX all-reduce
over xGMI combines them (MAX of 0/1 bytes = OR).  system_isolation reads one
row from the rank that owns it; policy_shadow's output is ordered by
container, so each rank emits its own rows' pairs and rank order is the
global order.
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
