"""Host interning: kano API objects -> the integer tables of include/kano_hip.h.

Semantics restated from the reference (kano_py/kano/model.py):

* KEYS = every label key carried by a container passed to build_matrix
  (the ``labelMap`` of model.py:127-133, a dict, so key equality is Python
  hash/==).
* A working-selector term (k, rule) whose key is not in KEYS is dropped: the
  presence AND skips it (model.py:143,146) and the refine loop never reaches it
  because it iterates the *container's* labels (model.py:95-111).  Quirk Q1.
* A kept term requires the pod to carry k (presence bitset) and
  ``matcher.match(rule, value)`` (model.py:66-68); with the default matcher
  that is ``rule == value`` (Python ==, so 1 == 1.0 == True).  Values are
  interned per key into equality classes with a dict; values that are not
  equal to themselves (NaN) never match and get a private id; unhashable
  values are matched by a linear == scan.
* Ingress policies swap the sides (working_selector = allow,
  model.py:82-93); that is read through the Policy properties themselves.
* A policy with a non-default matcher gets one virtual column per term: 1 where
  matcher.match(rule, value) holds, 0 where the pod carries the key but the
  matcher rejects, -1 where the pod lacks the key; the term becomes (column, 1).

Value id conventions: pod side -1 = key absent, -3 = never matches (NaN);
rule side -2 = no pod value equals the rule (matches nothing).
"""
from __future__ import annotations

from dataclasses import dataclass
from itertools import chain
from typing import Any, Dict, List, Sequence

import numpy as np

try:
    from . import _kano_host   # csrc/kano_hostext.c, built in-tree by __graft_entry__.build()
except ImportError:            # (missing or built for another interpreter ABI: the
    _kano_host = None          # Python loops below are the same steps, slower)

ABSENT = -1
NO_MATCH_RULE = -2
NEVER_MATCH_VALUE = -3


@dataclass
class Tables:
    n: int
    ncols: int
    pod_val: np.ndarray          # (ncols, n) int32
    sel_off: np.ndarray          # (P+1,) int64
    sel_col: np.ndarray
    sel_val: np.ndarray
    alw_off: np.ndarray
    alw_col: np.ndarray
    alw_val: np.ndarray
    # interning state of intern(): lets intern_more() put later policies in
    # the same id space (incremental updates)
    state: Any = None
    # matchExpressions requirements (model.LabelExpression): E columns the
    # engine appends after the ncols above (kano_set_expressions): base pod
    # column (-1: no container carries the key), operator, sorted value ids
    expr_col: Any = None
    expr_op: Any = None
    expr_off: Any = None
    expr_val: Any = None

    @property
    def P(self) -> int:
        return int(self.sel_off.shape[0] - 1)


class _ValueIndex:
    """Equality classes of one key's pod values under Python ==."""

    __slots__ = ("ids", "unhashable", "next_id")

    def __init__(self):
        self.ids: Dict[Any, int] = {}
        self.unhashable: List[tuple] = []
        self.next_id = 0

    def pod_id(self, v) -> int:
        try:
            if v != v:            # NaN-like: rule == v is False for every rule
                return NEVER_MATCH_VALUE
        except Exception:
            pass
        try:
            got = self.ids.get(v)
        except TypeError:
            for val, vid in self.unhashable:
                if val == v:
                    return vid
            vid = self.next_id
            self.next_id += 1
            self.unhashable.append((v, vid))
            return vid
        if got is None:
            got = self.next_id
            self.next_id += 1
            self.ids[v] = got
        return got

    def rule_id(self, rule) -> int:
        try:
            if rule != rule:
                return NO_MATCH_RULE
        except Exception:
            pass
        try:
            got = self.ids.get(rule)
        except TypeError:
            for val, vid in self.unhashable:
                if rule == val:
                    return vid
            return NO_MATCH_RULE
        return NO_MATCH_RULE if got is None else got


_MISSING = object()


def _intern_column(labels, k, idx: "_ValueIndex", row: np.ndarray) -> bool:
    """pod_id over one key's column at C speed (csrc/kano_hostext.c, the same
    steps per pod: v != v first, then the dict of equality classes, ids in
    first-seen order).  Returns False, idx untouched, when a value is
    unhashable (the per-pod loop handles it)."""
    if _kano_host is None:
        return False
    out = np.empty(len(labels), np.int32)
    ids: Dict[Any, int] = {}
    try:
        nxt = _kano_host.intern_column(labels, k, ids, out)
    except TypeError:
        return False
    idx.ids, idx.next_id = ids, nxt
    row[:] = out
    return True


def is_default_matcher(matcher) -> bool:
    from .model import DefaultEqualityLabelRelation
    return type(matcher).match is DefaultEqualityLabelRelation.match


def intern(containers: Sequence, policies: Sequence) -> Tables:
    n = len(containers)
    labels = [c.labels for c in containers]

    # working sides, read through the reference's own properties
    sides = [(pol.working_selector.labels, pol.working_allow.labels, pol.matcher)
             for pol in policies]

    # KEYS (first-seen order, as a nested loop over every label dict) and the
    # value-id columns of every key a policy term names, in one native pass
    # over the label dicts (csrc/kano_hostext.c scan_labels); non-dict label
    # maps or unhashable values: KEYS here, the columns one by one below
    # (a side that is not a mapping -- e.g. None, which the term loop below
    # reports as kano_py does -- leaves every column to that loop)
    try:
        cand = list(dict.fromkeys(chain.from_iterable(
            chain.from_iterable((ws, wa) for ws, wa, _ in sides))))
    except TypeError:
        cand = None
    scanned: Dict[Any, int] = {}
    scan_ids, scan_out = [], None
    keys: Dict[Any, None] = {}
    if _kano_host is None:
        cand = None
    if cand is not None:
        scan_ids = [{} for _ in cand]
        scan_out = np.empty((len(cand), n), np.int32)
        try:
            keys = _kano_host.scan_labels(labels, cand, scan_ids, scan_out)
            scanned = {k: j for j, k in enumerate(cand)}
        except (TypeError, ValueError):
            cand = None
    if cand is None:
        keys = dict.fromkeys(chain.from_iterable(labels))

    if scanned:
        t = _intern_fast(n, labels, keys, sides, scanned, scan_ids, scan_out)
        if t is not None:
            return t

    col_of_key: Dict[Any, int] = {}
    col_specs: List[tuple] = []          # ("key", k) or ("custom", k, rule, matcher)

    def key_col(k) -> int:
        c = col_of_key.get(k)
        if c is None:
            c = len(col_specs)
            col_of_key[k] = c
            col_specs.append(("key", k))
        return c

    from .model import LabelExpression
    exprs: List[tuple] = []              # (key, LabelExpression)
    raw_terms = []                       # per policy: ([(col, rule|None)], [(col, rule|None)])
    default_of: Dict[type, bool] = {}
    for ws, wa, matcher in sides:
        default = default_of.get(type(matcher))
        if default is None:
            default = default_of[type(matcher)] = is_default_matcher(matcher)
        per_side = []
        for side in (ws, wa):
            terms = []
            for k, rule in side.items():
                if isinstance(rule, LabelExpression):
                    # evaluated on the device from the key's column, whether or
                    # not a container carries the key (no quirk Q1)
                    if k in keys:
                        key_col(k)
                    terms.append((None, len(exprs), "expr"))
                    exprs.append((k, rule))
                    continue
                if k not in keys:
                    continue                 # quirk Q1
                if default:
                    terms.append((key_col(k), rule, False))
                else:
                    col = len(col_specs)
                    col_specs.append(("custom", k, rule, matcher))
                    terms.append((col, None, True))
            per_side.append(terms)
        raw_terms.append(per_side)

    ncols = len(col_specs)
    pod_val = np.full((ncols, n), ABSENT, dtype=np.int32)
    indexes: Dict[int, _ValueIndex] = {}
    plain = None
    for c, spec in enumerate(col_specs):
        row = pod_val[c]
        if spec[0] == "key":
            k = spec[1]
            idx = _ValueIndex()
            indexes[c] = idx
            j = scanned.get(k)
            if j is not None:
                row[:] = scan_out[j]
                idx.ids, idx.next_id = scan_ids[j], len(scan_ids[j])
                continue
            if plain is None:
                plain = all(type(lab) is dict for lab in labels)
            if not (plain and _intern_column(labels, k, idx, row)):
                for i, lab in enumerate(labels):
                    if k in lab:
                        row[i] = idx.pod_id(lab[k])
        else:
            _, k, rule, matcher = spec
            for i, lab in enumerate(labels):
                if k in lab:
                    row[i] = 1 if matcher.match(rule, lab[k]) else 0

    def csr(which: int):
        cnt = np.fromiter((len(per_side[which]) for per_side in raw_terms), np.int64,
                          count=len(raw_terms))
        off = np.zeros(len(raw_terms) + 1, dtype=np.int64)
        np.cumsum(cnt, out=off[1:])
        cols: List[int] = []
        vals: List[int] = []
        cadd, vadd = cols.append, vals.append
        for per_side in raw_terms:
            for col, rule, custom in per_side[which]:
                if custom == "expr":
                    cadd(ncols + rule)    # the engine's expression column
                    vadd(1)
                    continue
                cadd(col)
                vadd(1 if custom else indexes[col].rule_id(rule))
        return off, np.asarray(cols, dtype=np.int32), np.asarray(vals, dtype=np.int32)

    so, sc, sv = csr(0)
    ao, ac, av = csr(1)
    st = _InternState(labels, keys, col_of_key, indexes, ncols + len(exprs))
    t = Tables(n, ncols, pod_val, so, sc, sv, ao, ac, av, st)
    if exprs:
        ecol, eop, eoff, evals = [], [], [0], []
        for k, rule in exprs:
            c = col_of_key.get(k, -1) if k in keys else -1
            ecol.append(c)
            eop.append(rule.op)
            ids = set()
            if c >= 0:
                for v in getattr(rule, "values", ()):
                    vid = indexes[c].rule_id(v)
                    if vid >= 0:
                        ids.add(vid)
            evals.extend(sorted(ids))
            eoff.append(len(evals))
        t.expr_col = np.asarray(ecol, np.int32)
        t.expr_op = np.asarray(eop, np.int32)
        t.expr_off = np.asarray(eoff, np.int64)
        t.expr_val = np.asarray(evals, np.int32)
    return t


def _intern_fast(n, labels, keys, sides, scanned, scan_ids, scan_out):
    """intern's term loop in native code (csrc/kano_hostext.c policy_terms)
    when every matcher is the default equality and no term is a
    LabelExpression; None otherwise (intern's own loop then runs)."""
    from .model import LabelExpression
    if _kano_host is None:
        return None
    dflt: Dict[type, bool] = {}
    flags = [dflt[t] if (t := type(m)) in dflt else dflt.setdefault(t, is_default_matcher(m))
             for _, _, m in sides]
    try:
        col_keys, so, sc, sv, ao, ac, av = _kano_host.policy_terms(
            sides, flags, keys, scanned, scan_ids, LabelExpression)
    except LookupError:
        return None
    ncols = len(col_keys)
    rows = [scanned[k] for k in col_keys]
    pod_val = scan_out[rows] if ncols else np.zeros((0, n), np.int32)
    indexes: Dict[int, _ValueIndex] = {}
    for c, j in enumerate(rows):
        idx = _ValueIndex()
        idx.ids, idx.next_id = scan_ids[j], len(scan_ids[j])
        indexes[c] = idx
    col_of_key = {k: c for c, k in enumerate(col_keys)}
    arr = lambda b, d: np.frombuffer(b, dtype=d).copy()  # noqa: E731
    st = _InternState(labels, keys, col_of_key, indexes, ncols)
    return Tables(n, ncols, pod_val, arr(so, np.int64), arr(sc, np.int32), arr(sv, np.int32),
                  arr(ao, np.int64), arr(ac, np.int32), arr(av, np.int32), st)


class _InternState:
    __slots__ = ("labels", "keys", "col_of_key", "indexes", "ncols")

    def __init__(self, labels, keys, col_of_key, indexes, ncols):
        self.labels, self.keys, self.col_of_key = labels, keys, col_of_key
        self.indexes, self.ncols = indexes, ncols


def intern_more(t: Tables, policies: Sequence):
    """Working terms of further policies in the id space of intern()'s
    tables t (same KEYS, same value ids): returns (xval, sel CSR, allow CSR)
    where xval (ncols_x, n) holds the pod columns these policies add (keys no
    earlier policy used, custom-matcher columns), numbered after every column
    so far.  KEYS stay the build's (kano_py's labelMap, model.py:127-133)."""
    from .model import LabelExpression
    st = t.state
    if st is None:
        raise ValueError("tables without interning state (use intern())")
    n = t.n
    labels = st.labels
    new_cols: List[np.ndarray] = []

    def key_col(k) -> int:
        c = st.col_of_key.get(k)
        if c is None:
            c = st.ncols
            st.ncols += 1
            st.col_of_key[k] = c
            idx = _ValueIndex()
            st.indexes[c] = idx
            row = np.full(n, ABSENT, dtype=np.int32)
            for i, lab in enumerate(labels):
                if k in lab:
                    row[i] = idx.pod_id(lab[k])
            new_cols.append(row)
        return c

    sides = [[], []]
    for pol in policies:
        default = is_default_matcher(pol.matcher)
        for which, side in enumerate((pol.working_selector.labels, pol.working_allow.labels)):
            terms = []
            for k, rule in side.items():
                if isinstance(rule, LabelExpression):
                    c = st.ncols
                    st.ncols += 1
                    row = np.fromiter((1 if rule.matches(lab, k) else 0 for lab in labels),
                                      dtype=np.int32, count=n)
                    new_cols.append(row)
                    terms.append((c, 1))
                    continue
                if k not in st.keys:
                    continue                 # quirk Q1
                if default:
                    c = key_col(k)
                    terms.append((c, st.indexes[c].rule_id(rule)))
                else:
                    c = st.ncols
                    st.ncols += 1
                    row = np.full(n, ABSENT, dtype=np.int32)
                    for i, lab in enumerate(labels):
                        if k in lab:
                            row[i] = 1 if pol.matcher.match(rule, lab[k]) else 0
                    new_cols.append(row)
                    terms.append((c, 1))
            sides[which].append(terms)

    def csr(lists):
        off = np.zeros(len(lists) + 1, dtype=np.int64)
        np.cumsum([len(x) for x in lists], out=off[1:])
        cols = np.array([c for x in lists for c, _ in x], dtype=np.int32)
        vals = np.array([v for x in lists for _, v in x], dtype=np.int32)
        return off, cols, vals

    xval = np.stack(new_cols) if new_cols else np.zeros((0, n), np.int32)
    return xval, csr(sides[0]), csr(sides[1])


def tables_from_cluster(cl) -> Tables:
    """Direct tables of a synth.Cluster (no Python objects), restricted to the
    columns the working terms reference."""
    (so, sk, sv), (ao, ak, av) = cl.working_terms()
    used = sorted(set(sk.tolist()) | set(ak.tolist()))
    remap = {k: i for i, k in enumerate(used)}
    pod_val = np.ascontiguousarray(cl.vals[used], dtype=np.int32) if used else \
        np.zeros((0, cl.n), np.int32)
    rm = np.vectorize(remap.get, otypes=[np.int32]) if used else None
    sc = rm(sk) if sk.size else sk.astype(np.int32)
    ac = rm(ak) if ak.size else ak.astype(np.int32)
    return Tables(cl.n, len(used), pod_val, so, sc, sv.astype(np.int32), ao, ac,
                  av.astype(np.int32))


def group_ids(containers: Sequence, label) -> np.ndarray:
    """gid[i] = dense id of container.getValueOrDefault(label, "") under the
    dict semantics of user_hashmap (kano_py/kano/algorithm.py:20-24)."""
    from .model import Container
    n = len(containers)
    if n and type(containers) is list and _kano_host is not None:
        # (Container.getValueOrDefault is labels[key] if present, else the
        # default: the native loop does that for exact Containers with dict
        # labels, ids by first appearance as below; anything else -> the loop)
        gid = np.empty(n, dtype=np.int32)
        try:
            _kano_host.group_ids(containers, Container, label, gid)
            return gid
        except ValueError:
            pass
    groups: Dict[Any, int] = {}
    gid = np.empty(n, dtype=np.int32)
    for i, c in enumerate(containers):
        v = c.getValueOrDefault(label, "")
        g = groups.get(v)
        if g is None:
            g = len(groups)
            groups[v] = g
        gid[i] = g
    return gid
