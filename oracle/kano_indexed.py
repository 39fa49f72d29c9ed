"""TEST INFRASTRUCTURE ONLY -- an indexed restatement of kano_py's build and
checks for clusters whose matrix no list-based oracle can hold (C5: 10^6 pods,
a 125 GB matrix, ~10^11 pod pairs).

Imported by tests/ and tests/golden/make_c5.py; never by the product package,
and written without any of it (no kano._intern, no engine): its input is the
cluster's raw tables (``vals[k, i]`` value id of key k on pod i or -1, the
direction flags and the two per-policy term CSRs, key -1 = a key no pod
carries), i.e. what kano.synth generates before any interning.

The reference (kano_py/kano/model.py:125-165) builds, per policy p, a select
set and an allow set over the pods -- pod i is in the set iff, for every term
(k, v) of the working side whose key some pod carries, pod i carries k with
value v (select_set &= labelMap[k] at :142-147 makes the key required; the
value test of select_policy / allow_policy at :95-111 makes it equal; keys no
pod carries are skipped, quirk Q1) -- and ORs allow_p into row i of the matrix
for every p selecting i.  Both predicates read only the pod's values on keys
some working term names, so they are constant on the *classes* of pods with
equal values on those keys (plus the check label, so every class has one
tenant).  Everything below works on classes:

* Sel, Alw   policy x class incidence (a policy's set is a union of classes);
* R = Sel^T Alw > 0   class x class: row of any pod of class c is the union of
             the pods of the classes in R[c]; column j of class a is the union
             of the pods of the classes c with a in R[c];
* the Kano checks (kano_py/kano/algorithm.py:4-80) on those unions, and the
  row digests of kano_rows_digest (one per class, shared by its pods).

Pinned against kano_py's own records on C2 and C3 (tests/test_oracle_indexed.py:
M_sha256, the select / allow set shas, every check list and policy_shadow's
pairs sha256), then run on C5 by tests/golden/make_c5.py.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np
import scipy.sparse as sp

_MIX = (np.uint64(0x9e3779b97f4a7c15), np.uint64(0xbf58476d1ce4e5b9),
        np.uint64(0x94d049bb133111eb), np.uint64(0xD6E8FEB86659FD93))


def mix_words(w: np.ndarray, k: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of w ^ k * C (the per-word term of the row
    digest; tests/_golden.py:row_digest states the same formula)."""
    with np.errstate(over="ignore"):
        z = np.asarray(w, np.uint64) ^ (np.asarray(k, np.uint64) * _MIX[3])
        z = z + _MIX[0]
        z = (z ^ (z >> np.uint64(30))) * _MIX[1]
        z = (z ^ (z >> np.uint64(27))) * _MIX[2]
        return z ^ (z >> np.uint64(31))


@dataclass
class Indexed:
    n: int
    P: int
    cls: np.ndarray          # class of every pod (int64, n)
    size: np.ndarray         # pods per class
    label: np.ndarray        # the check label's value id per class (-1: absent -> "")
    order: np.ndarray        # pods sorted by class (stable: ascending pod index)
    start: np.ndarray        # order[start[c]:start[c+1]] = the pods of class c
    Sel: sp.csr_matrix       # P x C, 1 where policy p selects class c
    Alw: sp.csr_matrix       # P x C, 1 where policy p allows class c
    R: sp.csr_matrix         # C x C, row c = classes reachable from class c

    # ---- per-pod views --------------------------------------------------
    def pods_of(self, classes) -> np.ndarray:
        """Ascending pod indices of a set of classes."""
        classes = np.asarray(classes, np.int64)
        if classes.size == 0:
            return np.zeros(0, np.int64)
        parts = [self.order[self.start[c]:self.start[c + 1]] for c in classes]
        return np.sort(np.concatenate(parts))

    def row_bits(self, i: int) -> np.ndarray:
        """Row i of the matrix as n bools (model.py:158-160)."""
        c = self.cls[i]
        hit = np.zeros(self.size.shape[0], bool)
        hit[self.R.indices[self.R.indptr[c]:self.R.indptr[c + 1]]] = True
        return hit[self.cls]

    def row_words(self, i: int) -> np.ndarray:
        W = (self.n + 63) // 64
        buf = np.zeros(W * 64, np.uint8)
        buf[:self.n] = self.row_bits(i)
        return np.packbits(buf, bitorder="little").view("<u8")


def _terms(off, key, val, p, known) -> Tuple[Tuple[int, int], ...]:
    """The terms of one side that take part (model.py:142-147: keys no pod
    carries are skipped), sorted by key."""
    t = {}
    for j in range(off[p], off[p + 1]):
        k = int(key[j])
        if k >= 0 and known[k]:
            t[k] = int(val[j])
    return tuple(sorted(t.items()))


def build(vals: np.ndarray, ingress: np.ndarray, sel_csr, alw_csr, label_key: int) -> Indexed:
    """Classes, incidence and class reachability of kano_py's build_matrix
    (model.py:125-165) on the raw cluster tables.  ``sel_csr`` / ``alw_csr``
    are the policies' PolicySelect / PolicyAllow terms (off, key, val);
    ingress swaps them into the working sides (model.py:82-93)."""
    vals = np.asarray(vals, np.int32)
    K, n = vals.shape
    P = len(ingress)
    known = (vals >= 0).any(axis=1)
    ws, wa = [], []
    for p in range(P):
        s = _terms(*sel_csr, p, known)
        a = _terms(*alw_csr, p, known)
        if ingress[p]:           # working_selector = allow, working_allow = selector
            s, a = a, s
        ws.append(s)
        wa.append(a)
    used = sorted({k for side in (ws, wa) for t in side for k, _ in t} | {label_key})
    # pod classes: equal values on every key any working term names (+ label)
    if n:
        cv, cls = np.unique(vals[used].T, axis=0, return_inverse=True)
        cls = cls.reshape(-1).astype(np.int64)
    else:
        cv, cls = np.zeros((0, len(used)), np.int32), np.zeros(0, np.int64)
    C = cv.shape[0]
    col_of = {k: j for j, k in enumerate(used)}
    size = np.bincount(cls, minlength=C).astype(np.int64)
    order = np.argsort(cls, kind="stable")
    start = np.zeros(C + 1, np.int64)
    np.cumsum(size, out=start[1:])

    # a side's class set: the classes whose values equal the terms' values
    index: Dict[Tuple[int, ...], Tuple[np.ndarray, Dict[tuple, np.ndarray]]] = {}

    def classes_of(terms) -> np.ndarray:
        keys = tuple(k for k, _ in terms)
        if keys not in index:
            if keys:
                sub = cv[:, [col_of[k] for k in keys]]
                u, inv = np.unique(sub, axis=0, return_inverse=True)
                inv = inv.reshape(-1)
                srt = np.argsort(inv, kind="stable")
                bnd = np.concatenate([[0], np.cumsum(np.bincount(inv, minlength=u.shape[0]))])
                grp = {tuple(int(x) for x in u[g]): srt[bnd[g]:bnd[g + 1]]
                       for g in range(u.shape[0])}
            else:
                grp = {(): np.arange(C)}
            index[keys] = grp
        return index[keys].get(tuple(v for _, v in terms), np.zeros(0, np.int64))

    def incidence(side) -> sp.csr_matrix:
        rows, cols = [], []
        for p, t in enumerate(side):
            c = classes_of(t)
            rows.append(np.full(c.shape[0], p, np.int64))
            cols.append(c)
        r = np.concatenate(rows) if rows else np.zeros(0, np.int64)
        c = np.concatenate(cols) if cols else np.zeros(0, np.int64)
        m = sp.csr_matrix((np.ones(r.shape[0], np.int32), (r, c)), shape=(P, C))
        m.sort_indices()
        return m

    Sel = incidence(ws)
    Alw = incidence(wa)
    R = (Sel.T.tocsr() @ Alw).tocsr()
    R.data[:] = 1
    R.sort_indices()
    lab = cv[:, col_of[label_key]] if C else np.zeros(0, np.int32)
    return Indexed(n, P, cls, size, lab, order, start, Sel, Alw, R)


def build_cluster(cl, label_key: int = 0) -> Indexed:
    """kano.synth.Cluster (raw generator tables) -> Indexed."""
    return build(cl.vals, cl.ingress, (cl.pols_off, cl.pols_key, cl.pols_val),
                 (cl.pola_off, cl.pola_key, cl.pola_val), label_key)


# ---- the Kano checks (kano_py/kano/algorithm.py) ---------------------------
def column_classes(ix: Indexed):
    """Per class a: the covering classes of column j (any j in a), CSR."""
    return ix.R.T.tocsr()


def all_reachable(ix: Indexed, RT=None) -> np.ndarray:
    """algorithm.py:4-9: columns whose count is n."""
    RT = column_classes(ix) if RT is None else RT
    cover = RT @ ix.size
    return ix.pods_of(np.flatnonzero(cover == ix.n)) if ix.n else np.zeros(0, np.int64)


def all_isolated(ix: Indexed, RT=None) -> np.ndarray:
    """algorithm.py:12-17: empty columns."""
    RT = column_classes(ix) if RT is None else RT
    return ix.pods_of(np.flatnonzero(np.diff(RT.indptr) == 0))


def user_crosscheck(ix: Indexed, RT=None) -> np.ndarray:
    """algorithm.py:27-41: column j holds a pod whose label value differs
    from j's (a missing label reads as "", the -1 value here)."""
    RT = column_classes(ix) if RT is None else RT
    rows = np.repeat(np.arange(RT.shape[0]), np.diff(RT.indptr))
    other = ix.label[RT.indices] != ix.label[rows]
    hit = np.zeros(RT.shape[0], bool)
    hit[rows[other]] = True
    return ix.pods_of(np.flatnonzero(hit))


def system_isolation(ix: Indexed, idx: int) -> np.ndarray:
    """algorithm.py:44-53: the zeros of row idx."""
    return np.flatnonzero(~ix.row_bits(idx))


def select_lists(ix: Indexed) -> sp.csr_matrix:
    """Container.select_policies per class (model.py:161-162: policies in
    ascending order), C x P."""
    m = ix.Sel.T.tocsr()
    m.sort_indices()
    return m


def policy_shadow(ix: Indexed, want_sha: bool = True):
    """algorithm.py:58-80: for every pod i in order, every ordered pair
    (j, k), j != k, of its select list with allow_k a subset of allow_j.
    Returns (count, sha256 of the int32 (count, 2) array or None).

    Per class the pair list is computed once (policies with equal allow class
    sets share one subset test: |a & b| == |b| from one sparse product), then
    streamed into the hash in pod order."""
    SL = select_lists(ix)
    C = SL.shape[0]
    # distinct allow sets
    A = ix.Alw
    keys = [A.indices[A.indptr[p]:A.indptr[p + 1]].tobytes() for p in range(ix.P)]
    gid: Dict[bytes, int] = {}
    g_of = np.array([gid.setdefault(k, len(gid)) for k in keys], np.int64)
    G = len(gid)
    rep = np.zeros(G, np.int64)
    rep[g_of[::-1]] = np.arange(ix.P)[::-1]
    AG = A[rep]
    gsize = np.diff(AG.indptr)
    inter = (AG @ AG.T).tocsr()          # |a & b| where nonzero
    pair_bytes = [b""] * C
    pair_count = np.zeros(C, np.int64)
    memo: Dict[bytes, Tuple[int, bytes]] = {}
    for c in range(C):
        S = SL.indices[SL.indptr[c]:SL.indptr[c + 1]]
        if S.shape[0] < 2:
            continue
        key = S.tobytes()
        if key not in memo:
            g = g_of[S]
            ug, inv = np.unique(g, return_inverse=True)
            blk = inter[ug][:, ug].toarray()
            sub = blk == gsize[ug][None, :]          # sub[a, b]: allow_b <= allow_a
            sub |= (gsize[ug] == 0)[None, :]         # the empty set is in every set
            if not want_sha:
                # the count alone (D1: ~5e6 pairs per pod): sum over group
                # pairs of |a| |b| [allow_b <= allow_a], minus the j == k pairs
                cnt = np.bincount(inv, minlength=ug.shape[0]).astype(np.int64)
                memo[key] = (int(cnt @ sub.astype(np.int64) @ cnt) - S.shape[0], b"")
                pair_count[c] = memo[key][0]
                continue
            m = sub[inv][:, inv]
            np.fill_diagonal(m, False)
            jj, kk = np.nonzero(m)
            arr = np.stack([S[jj], S[kk]], axis=1).astype(np.int32)
            memo[key] = (arr.shape[0], arr.tobytes())
        pair_count[c], pair_bytes[c] = memo[key]
    total = int(pair_count[ix.cls].sum())
    if not want_sha:
        return total, None
    h = hashlib.sha256()
    for c in ix.cls.tolist():
        if pair_count[c]:
            h.update(pair_bytes[c])
    return total, h.hexdigest()


# ---- rows ------------------------------------------------------------------
def class_digests(ix: Indexed) -> np.ndarray:
    """kano_rows_digest of every class's row (the same for all its pods):
    sum_k mix(w_k ^ k*C) over the row's W words, computed as the all-zero
    row's sum plus, for the nonzero words only, mix(w) - mix(0-word)."""
    n = ix.n
    W = (n + 63) // 64
    kk = np.arange(W, dtype=np.uint64)
    zero_terms = mix_words(np.zeros(W, np.uint64), kk)
    with np.errstate(over="ignore"):
        base = zero_terms.sum(dtype=np.uint64)
    # pods of every class as (word, bit) once
    pw = (ix.order >> 6).astype(np.int64)
    pb = np.left_shift(np.uint64(1), (ix.order & 63).astype(np.uint64))
    C = ix.size.shape[0]
    out = np.empty(C, np.uint64)
    R = ix.R
    words = np.zeros(W, np.uint64)
    for c in range(C):
        targets = R.indices[R.indptr[c]:R.indptr[c + 1]]
        if targets.shape[0] == 0:
            out[c] = base
            continue
        sel = np.concatenate([np.arange(ix.start[t], ix.start[t + 1]) for t in targets])
        w_idx = pw[sel]
        np.bitwise_or.at(words, w_idx, pb[sel])
        nz = np.unique(w_idx)
        with np.errstate(over="ignore"):
            out[c] = base + (mix_words(words[nz], nz.astype(np.uint64)).sum(dtype=np.uint64)
                             - zero_terms[nz].sum(dtype=np.uint64))
        words[nz] = 0
    return out


def row_digests(ix: Indexed) -> np.ndarray:
    """Every row's digest, pod order (uint64, n)."""
    return class_digests(ix)[ix.cls]


def matrix_sha(ix: Indexed, chunk: int = 4096) -> str:
    """sha256 of the full matrix in the golden's canonical layout (row-major
    LSB-first uint64 words) -- for clusters up to ~10^5 pods."""
    n = ix.n
    W = (n + 63) // 64
    h = hashlib.sha256()
    rowc: Dict[int, bytes] = {}
    for i in range(n):
        c = int(ix.cls[i])
        if c not in rowc:
            rowc[c] = ix.row_words(i).tobytes()
        h.update(rowc[c])
        if len(rowc) > chunk:
            rowc.clear()
    if n == 0:
        h.update(np.zeros((0, W), np.uint64).tobytes())
    return h.hexdigest()


def set_words_sha(ix: Indexed, inc: sp.csr_matrix) -> str:
    """sha256 of the policies' select (or allow) sets as P rows of words
    (make_golden.py matrix_record's sel_sha256 / allow_sha256)."""
    n = ix.n
    W = (n + 63) // 64
    h = hashlib.sha256()
    for p in range(inc.shape[0]):
        cs = inc.indices[inc.indptr[p]:inc.indptr[p + 1]]
        hit = np.zeros(ix.size.shape[0], bool)
        hit[cs] = True
        buf = np.zeros(W * 64, np.uint8)
        buf[:n] = hit[ix.cls]
        h.update(np.packbits(buf, bitorder="little").view("<u8").tobytes())
    return h.hexdigest()


def lists_sha(ix: Indexed, inc: sp.csr_matrix) -> str:
    """sha256 of Container.select_policies (Sel) / allow_policies (Alw) for
    every pod as offsets int64 + indices int32 (make_golden.py csr)."""
    L = inc.T.tocsr()
    L.sort_indices()
    cnt = np.diff(L.indptr)[ix.cls]
    off = np.zeros(ix.n + 1, np.int64)
    np.cumsum(cnt, out=off[1:])
    parts: List[np.ndarray] = []
    for c in ix.cls.tolist():
        parts.append(L.indices[L.indptr[c]:L.indptr[c + 1]])
    flat = (np.concatenate(parts) if parts else np.zeros(0)).astype(np.int32)
    return hashlib.sha256(off.tobytes() + flat.tobytes()).hexdigest()


def list_record(lst) -> dict:
    a = np.ascontiguousarray(np.asarray(lst, np.int32))
    return {"count": int(a.shape[0]), "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
            "head": a[:64].tolist()}
