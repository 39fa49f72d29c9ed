"""TEST INFRASTRUCTURE ONLY -- the parity oracle.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg;
never by the product package.  Two layers:

* ``ref_py`` -- a pure-Python restatement of kano_py's build and checks that
  works on the kano API objects (dict labels, Python ==); for small clusters
  and the quirk cases (kano_py/kano/model.py:125-165,
  kano_py/kano/algorithm.py:4-100).
* ``run_c`` -- the same algorithm in C (oracle/kano_oracle.c, built into
  oracle/liboracle.so by oracle/Makefile) on integer tables produced by
  ``intern_json``, an interning written independently of the product's
  (kano/_intern.py), for clusters up to ~10^4 pods.

Both are pinned against tests/golden/, vectors produced by running kano_py
itself (tests/golden/make_golden.py, run under /opt/conda/bin/python3.9 in
the build container).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_int, c_int64, c_void_p
from typing import Any, Dict, List, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB)
        L.oracle_build.argtypes = [c_int64, c_int64] + [c_void_p] * 3 + [c_int64] + [c_void_p] * 9
        L.oracle_lists.argtypes = [c_int64, c_int64, c_void_p, c_void_p, c_void_p]
        L.oracle_column_checks.argtypes = [c_int64, c_void_p, c_int64, c_int64, c_void_p, c_void_p]
        L.oracle_crosscheck.argtypes = [c_int64, c_void_p, c_void_p, c_int64, c_int64, c_void_p]
        L.oracle_shadow.argtypes = [c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                                    c_int64, c_int64, c_void_p, POINTER(c_int64)]
        for f in (L.oracle_build, L.oracle_lists, L.oracle_column_checks, L.oracle_crosscheck,
                  L.oracle_shadow):
            f.restype = c_int
        L.oracle_path.argtypes = [c_int64, c_int64, c_void_p, c_int64, c_void_p]
        L.oracle_path.restype = c_int64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


# ---------------------------------------------------------------------------
# independent interning of a JSON cluster
# ---------------------------------------------------------------------------
def _eq_class(table: List[Tuple[Any, int]], index: Dict, v) -> int:
    """Equality class id of v under Python == (NaN never equal)."""
    if v != v:
        return -3
    try:
        hit = index.get(v)
    except TypeError:
        for w, cid in table:
            if w == v:
                return cid
        cid = len(table)
        table.append((v, cid))
        return cid
    if hit is None:
        hit = len(table)
        table.append((v, hit))
        index[v] = hit
    return hit


def intern_json(obj: dict):
    """cluster JSON -> label CSR + working term CSRs (key -1 = unknown key,
    value -2 = rule equal to no pod value)."""
    pods = obj["pods"]
    keys: Dict[Any, int] = {}
    for p in pods:
        for k in p["labels"]:
            keys.setdefault(k, len(keys))
    vtable: List[Tuple[Any, int]] = []
    vindex: Dict = {}
    lab_off = [0]
    lab_key: List[int] = []
    lab_val: List[int] = []
    for p in pods:
        for k, v in p["labels"].items():
            lab_key.append(keys[k])
            lab_val.append(_eq_class(vtable, vindex, v))
        lab_off.append(len(lab_key))

    def rule_id(r):
        if r != r:
            return -2
        try:
            hit = vindex.get(r)
            return -2 if hit is None else hit
        except TypeError:
            for w, cid in vtable:
                if w == r:
                    return cid
            return -2

    rcache: Dict = {}

    def rid(r):
        try:
            if r in rcache:
                return rcache[r]
            x = rule_id(r)
            rcache[r] = x
            return x
        except TypeError:
            return rule_id(r)

    def terms(side_of):
        off, ks, vs = [0], [], []
        for q in obj["policies"]:
            d = side_of(q)
            for k, r in d.items():
                ks.append(keys.get(k, -1))
                vs.append(rid(r))
            off.append(len(ks))
        return np.array(off, np.int64), np.array(ks, np.int32), np.array(vs, np.int32)

    def ws(q):  # working selector (model.py:82-87)
        return q["allow"] if q["direction"] == "ingress" else q["select"]

    def wa(q):  # working allow (model.py:89-93)
        return q["select"] if q["direction"] == "ingress" else q["allow"]

    return (len(pods), len(keys), np.array(lab_off, np.int64), np.array(lab_key, np.int32),
            np.array(lab_val, np.int32), len(obj["policies"]), terms(ws), terms(wa))


def group_ids_json(obj: dict, label) -> np.ndarray:
    groups: Dict = {}
    out = []
    for p in obj["pods"]:
        v = p["labels"].get(label, "")
        out.append(groups.setdefault(v, len(groups)))
    return np.array(out, np.int32)


def run_c(obj: dict, label="tenant", sys_idx=0, shadow_cap=10_000_000,
          policies=None) -> dict:
    """Full reference pipeline on a JSON cluster through the C restatement."""
    L = lib()
    n, K, lo, lk, lv, P, (so, sk, sv), (ao, ak, av) = intern_json(obj)
    if policies is not None:
        P = policies
        so, ao = so[: P + 1], ao[: P + 1]
    W = (n + 63) // 64
    M = np.zeros(max(n * W, 1), np.uint64)
    sel = np.zeros(max(P * W, 1), np.uint64)
    alw = np.zeros(max(P * W, 1), np.uint64)
    rc = L.oracle_build(n, K, _p(lo), _p(lk), _p(lv), P, _p(so), _p(sk), _p(sv), _p(ao), _p(ak),
                        _p(av), _p(M), _p(sel), _p(alw))
    assert rc == 0
    res = dict(n=n, P=P, W=W, M=M[: n * W].reshape(n, W), sel=sel[: P * W].reshape(P, W),
               allow=alw[: P * W].reshape(P, W))
    for name, sets in (("select", sel), ("allow", alw)):
        off = np.zeros(n + 1, np.int64)
        L.oracle_lists(n, P, _p(sets), _p(off), None)
        lst = np.zeros(max(int(off[-1]), 1), np.int32)
        L.oracle_lists(n, P, _p(sets), _p(off), _p(lst))
        res[name + "_off"], res[name + "_list"] = off, lst[: int(off[-1])]
    reach = np.zeros(max(n, 1), np.uint8)
    isol = np.zeros(max(n, 1), np.uint8)
    L.oracle_column_checks(n, _p(M), 0, n, _p(reach), _p(isol))
    res["all_reachable"] = np.flatnonzero(reach[:n]).tolist()
    res["all_isolated"] = np.flatnonzero(isol[:n]).tolist()
    gid = group_ids_json(obj, label)
    cross = np.zeros(max(n, 1), np.uint8)
    L.oracle_crosscheck(n, _p(M), _p(gid), 0, n, _p(cross))
    res["user_crosscheck"] = np.flatnonzero(cross[:n]).tolist()
    if n:
        row = res["M"][sys_idx]
        bits = np.unpackbits(row.view(np.uint8), bitorder="little")[:n]
        res["system_isolation"] = np.flatnonzero(bits == 0).tolist()
    else:
        res["system_isolation"] = []
    cnt = c_int64()
    out = np.zeros(2 * max(1, min(shadow_cap, 1)), np.int32)
    L.oracle_shadow(n, n, _p(res["select_off"]), _p(res["select_list"]), _p(alw), 0, n, 0, None,
                    ctypes.byref(cnt))
    total = int(cnt.value)
    out = np.zeros(2 * max(1, min(total, shadow_cap)), np.int32)
    L.oracle_shadow(n, n, _p(res["select_off"]), _p(res["select_list"]), _p(alw), 0, n,
                    min(total, shadow_cap), _p(out), ctypes.byref(cnt))
    res["shadow_count"] = total
    res["shadow"] = out[: 2 * min(total, shadow_cap)].reshape(-1, 2)
    res["conflict_raises"] = bool(n and np.diff(res["select_off"]).max(initial=0) >= 2)
    return res


# ---------------------------------------------------------------------------
# pure-Python restatement on kano API objects (small clusters, quirk cases)
# ---------------------------------------------------------------------------
def ref_py(containers, policies, label="app", sys_idx=0) -> dict:
    """kano_py semantics restated with sets of ints; returns the matrix as a
    list of 0/1 strings and every check.  kano_py/kano/model.py:125-165 and
    algorithm.py:4-100."""
    n = len(containers)
    keys = set()
    for c in containers:
        keys.update(c.labels.keys())                       # model.py:131-133
    M = [[0] * n for _ in range(n)]
    sel_sets, alw_sets = [], []
    sel_lists = [[] for _ in range(n)]
    alw_lists = [[] for _ in range(n)]

    def is_expr(rule):   # a matchExpressions requirement (extension)
        return hasattr(rule, "matches")

    def expr_ok(pol_labels, cl):
        # K8s label-selector requirements (kubesv/kubesv/model.py:127-160):
        # In: key present, value listed; NotIn: absent or unlisted; Exists;
        # DoesNotExist.  Python == for values.
        for k, r in pol_labels.items():
            if not is_expr(r):
                continue
            name = type(r).__name__
            present = k in cl
            listed = present and any(cl[k] == x for x in getattr(r, "values", ()))
            ok = {"In": listed, "NotIn": not listed, "Exists": present,
                  "DoesNotExist": not present}[name]
            if not ok:
                return False
        return True

    def pred(pol_labels, cl, matcher):                      # model.py:95-111
        for k, v in cl.items():
            if k in pol_labels.keys() and not is_expr(pol_labels[k]) and \
                    not matcher.match(pol_labels[k], v):
                return False
        return expr_ok(pol_labels, cl)

    for p, pol in enumerate(policies):
        ws = pol.working_selector.labels                    # model.py:82-93
        wa = pol.working_allow.labels
        s = [int(all(k in c.labels for k in ws if k in keys and not is_expr(ws[k])))
             for c in containers]
        a = [int(all(k in c.labels for k in wa if k in keys and not is_expr(wa[k])))
             for c in containers]
        for i, c in enumerate(containers):                  # model.py:150-154
            if s[i] and not pred(ws, c.labels, pol.matcher):
                s[i] = 0
            if a[i] and not pred(wa, c.labels, pol.matcher):
                a[i] = 0
        sel_sets.append(s)
        alw_sets.append(a)
        for i in range(n):                                  # model.py:158-163
            if s[i]:
                M[i] = [x | y for x, y in zip(M[i], a)]
                sel_lists[i].append(p)
            if a[i]:
                alw_lists[i].append(p)

    def col(j):
        return [M[i][j] for i in range(n)]

    groups = {}
    g = []
    for c in containers:
        v = c.getValueOrDefault(label, "")
        g.append(groups.setdefault(v, len(groups)) if _hashable(v) else id(v))
    res = {
        "M": ["".join(map(str, r)) for r in M],
        "sel": ["".join(map(str, s)) for s in sel_sets],
        "allow": ["".join(map(str, a)) for a in alw_sets],
        "select_policies": sel_lists,
        "allow_policies": alw_lists,
        "all_reachable": [j for j in range(n) if sum(col(j)) == n],
        "all_isolated": [j for j in range(n) if sum(col(j)) == 0],
        "user_crosscheck": [j for j in range(n)
                            if any(col(j)[i] and g[i] != g[j] for i in range(n))],
        "system_isolation": [j for j in range(n) if not M[sys_idx][j]] if n else [],
    }
    pairs = []
    for i in range(n):                                      # algorithm.py:66-79
        for j in sel_lists[i]:
            for k in sel_lists[i]:
                if j == k:
                    continue
                if all(alw_sets[j][x] or not alw_sets[k][x] for x in range(n)):
                    pairs.append((j, k))
    res["policy_shadow"] = pairs
    res["conflict_raises"] = any(len(l) >= 2 for l in sel_lists)
    return res


def _hashable(v) -> bool:
    try:
        hash(v)
        return True
    except TypeError:
        return False


# ---------------------------------------------------------------------------
# multi-hop reachability (kubesv/kubesv/constraint.py:233-237)
def path_c(M: np.ndarray, n: int, hops: int = 2):
    """kubesv's `path` over kano's matrix (oracle_path): P = M | M.M for
    hops=2, paths of <= hops edges, or the transitive closure for hops=0.
    M: (n, W) uint64 LSB-first rows.  Returns (P, steps)."""
    M = np.ascontiguousarray(M, dtype=np.uint64)
    W = M.shape[1] if M.ndim == 2 else 0
    P = np.zeros_like(M)
    steps = lib().oracle_path(n, W, _p(M), int(hops), _p(P))
    if steps < 0:
        raise MemoryError("oracle_path")
    return P, int(steps)


def path_py(edges: set, n: int, hops: int = 2) -> set:
    """The Datalog rules of kubesv/kubesv/constraint.py:233-237 restated on
    sets of (src, dst) pairs, for tiny cases: path :- edge; path :- edge o
    edge (hops=2), extended to <= hops edges or to the closure (hops=0)."""
    succ = {}
    for a, b in edges:
        succ.setdefault(a, set()).add(b)
    path = set(edges)
    k = 1
    while hops == 0 or k < hops:
        new = {(a, c) for (a, b) in path for c in succ.get(b, ())} | set(edges)
        new |= path
        k += 1
        if new == path:
            break
        path = new
    return path


# ---------------------------------------------------------------------------
# kubesv's Kubernetes relations, restated on Python
# sets straight from the Datalog rules -- independent of kano/k8s.py's
# compilation to kano policies.  Unpinned: kubesv needs z3 and the kubernetes
# client, both absent.  Inputs are the kano.k8s objects (name / namespace /
# labels, NetworkPolicy.spec dicts).
# ---------------------------------------------------------------------------

def _k8s_selector(selector, known: set):
    """LabelSelectorAdapter.define_label_selector (kubesv/kubesv/model.py:
    178-233) as a predicate over a labels dict, or None on a quick fail."""
    if selector is None:
        return lambda lab: True
    reqs = []
    exprs = selector.get("matchExpressions")
    if exprs is not None:
        for e in exprs:                                   # model.py:139-158
            op = str(e.get("operator", "")).lower()
            if op not in ("in", "notin", "exists", "doesnotexists"):
                continue
            if e.get("key") not in known:
                return None
            reqs.append((op, e["key"], list(e.get("values") or [])))
    labels = selector.get("matchLabels")
    if labels is not None:
        for k, v in labels.items():
            if k not in known:
                return None
            reqs.append(("in", k, [v]))

    def pred(lab):
        for op, k, vals in reqs:
            has = k in lab
            listed = has and any(lab[k] == v for v in vals)
            if op == "in" and not listed:
                return False
            if op == "notin" and listed:
                return False
            if op == "exists" and not has:
                return False
            if op == "doesnotexists" and has:
                return False
        return True
    return pred


def kubesv_edge_py(pods, policies, namespaces, check_self_ingress_traffic=True,
                   check_select_by_no_policy=False):
    """edge(src, dst) as a set of pairs (kubesv/kubesv/constraint.py:168-231),
    with the facts of define_pod_facts (:242-275) and define_pol_facts
    (:278-282, model.py:420-514)."""
    nam_map = {ns.name: i for i, ns in enumerate(namespaces)}
    ns_lab = {ns.name: ns.labels for ns in namespaces}
    pod_ns = [nam_map[p.namespace] for p in pods]       # KeyError as :251
    del pod_ns
    pod_keys = {k for p in pods for k in p.labels}
    ns_keys = {k for ns in namespaces for k in ns.labels}
    n = len(pods)
    selected_by_pol = set()                             # (pod, pol)
    ingress_allow, egress_allow = set(), set()          # (pod, pol)
    for idx, pol in enumerate(policies):
        spec = pol.spec
        # define_pod_selector (model.py:496-514)
        if pol.namespace in nam_map:
            pred = _k8s_selector(spec.get("podSelector"), pod_keys)
            if pred is not None:
                for i, p in enumerate(pods):
                    if p.namespace == pol.namespace and pred(p.labels):
                        selected_by_pol.add((i, idx))

        def rules(direction, key, out):
            for rule in spec.get(direction):
                for peer in (rule or {}).get(key):
                    peer = peer or {}
                    nsp = _k8s_selector(peer.get("namespaceSelector"), ns_keys)
                    if nsp is None:
                        continue
                    pp = _k8s_selector(peer.get("podSelector"), pod_keys)
                    if pp is None:
                        continue
                    for i, p in enumerate(pods):   # namespace(pod, ns), ns free
                        if nsp(ns_lab[p.namespace]) and pp(p.labels):
                            out.add((i, idx))
        # define_egress_rules (model.py:420-437)
        if spec.get("egress") is not None:
            rules("egress", "to", egress_allow)
        # define_ingress_rules (model.py:466-483): guarded by egress
        if spec.get("egress") is not None:
            rules("ingress", "from", ingress_allow)
    pols_of = {}
    for (i, q) in selected_by_pol:
        pols_of.setdefault(i, set()).add(q)
    ing_by = {}
    for (i, q) in ingress_allow:
        ing_by.setdefault(q, set()).add(i)
    eg_by = {}
    for (i, q) in egress_allow:
        eg_by.setdefault(q, set()).add(i)
    # ingress_traffic(src, sel), egress_traffic(dst, sel) (constraint.py:191-227)
    ingress = {s: set() for s in range(n)}              # sel -> srcs
    egress = {s: set() for s in range(n)}               # sel -> dsts
    for s in range(n):
        for q in pols_of.get(s, ()):
            ingress[s] |= ing_by.get(q, set())
            egress[s] |= eg_by.get(q, set())
        if check_self_ingress_traffic:
            ingress[s].add(s)
        if check_select_by_no_policy and s not in pols_of:
            ingress[s] = set(range(n))
            egress[s] = set(range(n))
    # edge(src, dst) :- ingress_traffic(src, sel), egress_traffic(dst, sel)
    edge = set()
    for s in range(n):
        for src in ingress[s]:
            for dst in egress[s]:
                edge.add((src, dst))
    return edge, ingress, egress


# ---------------------------------------------------------------------------
# policy_shadow's pair count where the list itself is out of reach
def shadow_count_grouped(obj: dict) -> int:
    """len(policy_shadow(m, policies, containers)) (kano_py/kano/
    algorithm.py:58-80) without materialising the pairs: the reference
    appends (j, k) for every pod i and every ordered pair j != k of
    containers[i].select_policies with allow_k a subset of allow_j.  The
    count is restated as

        sum over row classes c of  m_c * sum_{j != k in S(c)} [allow_k <= allow_j]

    where a row class is the set of pods with equal values on every key a
    working selector names (the predicate of model.py:95-111 and the
    presence AND of :142-147 read nothing else, so S is constant on it) and
    policies with equal allow sets share one subset test.  Interning is the
    oracle's own (intern_json); allow sets come from the predicate of
    model.py:104-111 / :145-147 evaluated on the pod value table.  Pinned
    against kano_py's own counts (tests/test_oracle_golden.py); used for C4,
    whose ~1e11 pairs no list holds."""
    n, K, lo, lk, lv, P, (so, sk, sv), (ao, ak, av) = intern_json(obj)
    V = np.full((max(K, 1), n), -1, np.int32)
    V[lk, np.repeat(np.arange(n), np.diff(lo))] = lv
    W = (n + 63) // 64
    A = np.zeros((P, W), np.uint64)
    for p in range(P):
        m = np.ones(n, bool)
        for t in range(ao[p], ao[p + 1]):
            if ak[t] >= 0:                       # unknown keys are ignored (Q1)
                m &= V[ak[t]] == av[t]
        buf = np.zeros(W * 64, np.uint8)
        buf[:n] = m
        A[p] = np.packbits(buf, bitorder="little").view("<u8")
    R, g_of = np.unique(A, axis=0, return_inverse=True)
    g_of = g_of.reshape(-1)
    G = R.shape[0]
    sub = np.full((G, G), -1, np.int8)          # sub[a, b] = R[b] <= R[a], filled lazily
    keys = np.unique(sk[sk >= 0])
    if keys.size:
        _, rep, m_c = np.unique(V[keys].T, axis=0, return_index=True, return_counts=True)
    else:
        rep, m_c = np.array([0] if n else [], np.int64), np.array([n] if n else [], np.int64)
    total = 0
    for i, mc in zip(rep.tolist(), m_c.tolist()):
        ok = (sk < 0) | (V[np.maximum(sk, 0), i] == sv)
        cs = np.concatenate([[0], np.cumsum(~ok)])
        S = np.flatnonzero(cs[so[1:]] - cs[so[:-1]] == 0)
        if S.size < 2:
            continue
        gs, cnt = np.unique(g_of[S], return_counts=True)
        blk = sub[np.ix_(gs, gs)]
        for ai in np.flatnonzero((blk < 0).any(axis=1)):
            a = gs[ai]
            sub[a, gs] = ~np.any(R[gs] & ~R[a], axis=1)
        blk = sub[np.ix_(gs, gs)].astype(np.int64)
        cnt = cnt.astype(np.int64)
        total += mc * (int(cnt @ blk @ cnt) - int(S.size))
    return int(total)
