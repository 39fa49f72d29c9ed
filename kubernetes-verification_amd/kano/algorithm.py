"""Kano verification queries, drop-in for ``kano.algorithm`` of kano_py.

Every query runs on the device-resident matrix (kano/_engine.py ->
libkano_hip.so) and returns the reference's Python types: ascending
``List[int]`` index lists and a ``List[Tuple[int, int]]`` for policy_shadow.
Reference: kano_py/kano/algorithm.py:4-100.
"""
from __future__ import annotations

from typing import DefaultDict, Dict, List, Tuple

import numpy as np

from .model import *  # noqa: F401,F403  (the reference does the same, algorithm.py:1)
from .model import BitArray, Container, Policy, ReachabilityMatrix
from ._bits import bool_to_words, set_bit_indices, words_to_bool
from ._intern import group_ids
try:
    from . import _kano_host   # csrc/kano_hostext.c (host-side loops, no GPU work)
except ImportError:            # (missing or built for another interpreter: the
    _kano_host = None          # Python loops below do the same work)


def _engine(matrix: ReachabilityMatrix, whole: bool = True):
    """The matrix's device context.  A context holding only a row shard
    (a multi-GPU rank's rows) cannot answer a whole-matrix query on its own:
    the column checks, getcol and policy_shadow need every row, so they raise
    instead of returning the shard's part (combine shards with
    kano.shard.ShardExchange)."""
    eng = getattr(matrix, "_engine", None)
    if eng is None:
        raise TypeError("expected a kano ReachabilityMatrix built by this package")
    if whole and getattr(eng, "is_shard", False):
        r0, r1 = eng.row_span
        raise ValueError(f"matrix holds only rows [{r0}, {r1}) of {matrix.container_size}: "
                         "whole-matrix checks need every row (combine the row shards "
                         "with kano.shard.ShardExchange)")
    return eng


def all_reachable(matrix: ReachabilityMatrix) -> List[int]:
    """Columns j with M[i, j] = 1 for every row i (algorithm.py:4-9)."""
    eng = _engine(matrix)
    n = matrix.container_size
    if n == 0:
        return []
    col_and, _ = eng.col_checks()
    return set_bit_indices(col_and, n).tolist()


def all_isolated(matrix: ReachabilityMatrix) -> List[int]:
    """Columns j with M[i, j] = 0 for every row i (algorithm.py:12-17)."""
    eng = _engine(matrix)
    n = matrix.container_size
    if n == 0:
        return []
    _, col_or = eng.col_checks()
    return np.flatnonzero(~words_to_bool(col_or, n)).tolist()


def user_hashmap(containers: List[Container], label: str) -> Dict[str, BitArray]:
    """Group bitsets keyed by container.getValueOrDefault(label, "")
    (algorithm.py:20-24)."""
    n = len(containers)
    gid = group_ids(containers, label)
    keys: Dict = {}
    for c in containers:
        keys.setdefault(c.getValueOrDefault(label, ""), None)
    out: Dict = DefaultDict(lambda: BitArray(n))
    for g, key in enumerate(keys):
        out[key] = BitArray.from_words(bool_to_words(gid == g), n)
    return out


def user_crosscheck(matrix: ReachabilityMatrix, containers: List[Container],
                    label: str) -> List[int]:
    """Containers j reachable from a container of another user group
    (algorithm.py:27-42): j such that M[i, j] and g(i) != g(j) for some i."""
    eng = _engine(matrix)
    n = matrix.container_size
    if len(containers) != n:
        # the reference indexes user_map bitsets (len(containers) bits) with
        # columns of the matrix: mismatched sizes raise there as well
        raise ValueError("bitarrays of equal length expected for bitwise operation")
    if n == 0:
        return []
    gid = group_ids(containers, label)
    cross = eng.crosscheck(gid)
    return set_bit_indices(cross, n).tolist()


def system_isolation(matrix: ReachabilityMatrix, idx: int) -> List[int]:
    """Containers j not reachable from container idx (algorithm.py:45-55).
    On a row shard, idx must be one of the shard's rows."""
    eng = _engine(matrix, whole=False)
    n = matrix.container_size
    i = int(idx)
    if i < 0:
        i += n
    if not 0 <= i < n:
        raise IndexError("list index out of range")
    row = eng.rows(i, 1)[0]
    return np.flatnonzero(~words_to_bool(row, n)).tolist()


def _pairs_to_list(pairs: np.ndarray, P: int = 0) -> List[Tuple[int, int]]:
    if pairs.shape[0] == 0:
        return []
    # (csrc/kano_hostext.c: the tuples built natively, policy ints shared)
    if _kano_host is None:
        return [tuple(p) for p in pairs.tolist()]
    return _kano_host.pairs_list(np.ascontiguousarray(pairs, dtype=np.int32), int(P))


def _fast_path(matrix, policies, containers) -> bool:
    """True when (policies, containers) are exactly what this matrix's build
    saw and every container's select_policies is still that build's list."""
    if getattr(matrix, "_lists", None) is None:
        return False
    if matrix._policies is not policies and list(matrix._policies) != list(policies):
        return False
    if len(containers) != matrix._ncontainers:
        return False
    lists = matrix._lists
    order = lists._containers        # (the build's container order, snapshotted)
    if (_kano_host is not None and type(containers) is list and type(order) is list and
            _kano_host.pending_is(containers, Container, lists, order)):
        return True                  # (the loop below, natively, for exact Containers)
    if len(order) != len(containers):
        return False
    for c, o in zip(containers, order):
        if not isinstance(c, Container) or c is not o:
            return False
        if c._sel or len(c._pending) != 1 or c._pending[0] is not lists:
            return False
    return True


def policy_shadow_pairs(matrix: ReachabilityMatrix, policies: List[Policy],
                        containers: List[Container]) -> np.ndarray:
    """policy_shadow as an (T, 2) int32 array (compact form, same order)."""
    if _fast_path(matrix, policies, containers):
        return _engine(matrix).shadow()
    # general form: explicit per-container lists (accumulated builds, edited
    # lists) and each policy's current working_allow_set
    from ._engine import shadow_from_lists
    lists = [list(c.select_policies) for c in containers]
    soff = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum([len(l) for l in lists], out=soff[1:])
    flat = np.fromiter((x for l in lists for x in l), dtype=np.int64, count=int(soff[-1]))
    P = len(policies)
    if flat.size and (flat.min() < 0 or flat.max() >= P):
        raise IndexError("list index out of range")
    needed = np.unique(flat) if flat.size else np.zeros(0, np.int64)
    nbits = None
    for p in needed.tolist():
        s = policies[p].working_allow_set
        if s is None:
            raise AttributeError("'NoneType' object has no attribute '__and__'")
        if nbits is None:
            nbits = len(s)
        elif len(s) != nbits:
            raise ValueError("bitarrays of equal length expected for bitwise operation")
    nbits = nbits or 0
    W = (nbits + 63) >> 6
    aw = np.zeros((P, W), dtype=np.uint64)
    for p in needed.tolist():
        s = policies[p].working_allow_set
        b = s if isinstance(s, BitArray) else BitArray(s)
        aw[p] = b.words()[:W]
    return shadow_from_lists(len(lists), nbits, soff, flat.astype(np.int32), aw,
                             device=_engine(matrix).device)


def policy_shadow(matrix: ReachabilityMatrix, policies: List[Policy],
                  containers: List[Container]) -> List[Tuple[int, int]]:
    """Pairs (j, k) of policies selecting a common container with allow_k a
    subset of allow_j, one entry per container, in container order
    (algorithm.py:58-80; duplicates kept, quirk Q4)."""
    return _pairs_to_list(policy_shadow_pairs(matrix, policies, containers), len(policies))


def policy_conflict(matrix: ReachabilityMatrix, policies: List[Policy],
                    containers: List[Container]) -> List[Tuple[int, int]]:
    """Reproduces algorithm.py:83-100 as written: the loop binds ``pj`` to a
    policy *index*, so the first container with two selecting policies raises
    ``AttributeError`` (quirk Q3); otherwise the result is []."""
    if _fast_path(matrix, policies, containers):
        raises = _engine(matrix).conflict_raises()
    else:
        raises = any(len(c.select_policies) >= 2 for c in containers)
    if raises:
        raise AttributeError("'int' object has no attribute 'working_allow_set'")
    return []


# ---------------------------------------------------------------------------
# Multi-hop reachability.  Not part of kano_py's
# algorithm.py: kubesv's `path` relation (kubesv/kubesv/constraint.py:233-237,
# path(src, dst) :- edge(src, dst); path(src, dst) :- edge(src, sel),
# edge(sel, dst)) with kano's matrix as `edge`.  The result is a
# ReachabilityMatrix on the device, so every query above runs on it.

def _path_matrix(matrix: ReachabilityMatrix, hops: int, mode: str) -> ReachabilityMatrix:
    from ._engine import DeviceBuild
    from .multi import MultiBuild
    src = _engine(matrix)
    n = matrix.container_size
    out = ReachabilityMatrix.__new__(ReachabilityMatrix)
    out.container_size = n
    # a row-sharded group's path matrix is sharded the same way
    out._engine = (MultiBuild.empty(n, src.G, devices=src.devices)
                   if isinstance(src, MultiBuild) else DeviceBuild.empty(n, device=src.device))
    out._containers = None
    out._policies = None
    out._ncontainers = n
    out._lists = None
    out.path_info = out._engine.path_from(src, hops=hops, mode=mode)
    return out


def two_hop(matrix: ReachabilityMatrix, mode: str = "auto") -> ReachabilityMatrix:
    """kubesv's path relation: P = M | M.M (pairs joined by one or two
    edges)."""
    return _path_matrix(matrix, 2, mode)


def k_hop(matrix: ReachabilityMatrix, hops: int, mode: str = "auto") -> ReachabilityMatrix:
    """Pairs joined by a path of at most `hops` (>= 1) edges."""
    if int(hops) < 1:
        raise ValueError("hops must be >= 1")
    return _path_matrix(matrix, int(hops), mode)


def transitive_closure(matrix: ReachabilityMatrix, mode: str = "auto") -> ReachabilityMatrix:
    """M+: pairs joined by a path of any length >= 1 (the fixpoint of the
    path rule applied to itself)."""
    return _path_matrix(matrix, 0, mode)
