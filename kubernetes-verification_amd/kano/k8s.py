"""kubesv's Kubernetes reading of NetworkPolicies, on kano's engine
(namespaces, namespaceSelector, per-direction rules,
self traffic and pods selected by no policy).

kano_py reads a policy as one (select, allow) pair of equality selectors.
kubesv (kubesv/kubesv/model.py, constraint.py) reads Kubernetes objects:

* ``selected_by_pol(pod, pol)`` -- pod in the policy's namespace matching its
  ``podSelector`` (model.py:496-514);
* ``ingress_allow_by_pol`` / ``egress_allow_by_pol(pod, pol)`` -- pod matching
  one peer of one rule: ``namespaceSelector`` on the pod's namespace's labels,
  ``podSelector`` on the pod's labels (model.py:296-307,349-362,420-483);
* ``ingress_traffic(src, sel)``, ``egress_traffic(dst, sel)``,
  ``edge(src, dst) :- ingress_traffic(src, sel), egress_traffic(dst, sel)``
  and ``path`` (constraint.py:168-237).

Here each (policy, peer) becomes one kano policy: select = the policy's pod
selector and namespace, allow = the peer's terms -- matchLabels as plain kano
values (the quick fail guarantees some pod carries the key, so kano's quirk
Q1 cannot fire), matchExpressions as requirement columns (``model.In``
etc.).  Two device builds give
InT[sel][src] and EgT[sel][dst]; ``kano_k8s_edge`` forms the edge matrix on
the device (kano_k8s.hpp).  Every check of ``kano.algorithm`` and the path
functions then read it like any matrix.

kubesv's behaviour is kept where it departs from the Kubernetes documents
(each was read off the code):

* K1 a peer's ``podSelector`` without ``namespaceSelector`` matches pods of
  every namespace (the ``namespace(pod, ns)`` atom leaves ``ns`` free,
  model.py:435-436);
* K2 a selector naming a label key no pod (for ``namespaceSelector``: no
  namespace) carries fails as a whole -- the policy selects nothing, the
  peer matches nothing (model.py:196-201,224-232, "quick fail");
* K3 matchExpressions operators compare lower-cased against ``in``,
  ``notin``, ``exists``, ``doesnotexists``; anything else (Kubernetes'
  ``DoesNotExist`` included) is dropped (model.py:149-156);
* K4 ingress rules count only when the policy also has ``egress``
  (model.py:474-476); ``ingress: null`` beside an ``egress`` list, and a rule
  whose ``from`` / ``to`` is null, raise ``TypeError`` (iterating None,
  model.py:478,436 via :352-356);
* K5 a peer with neither selector (an ``ipBlock``) matches every pod
  (model.py:296-307: no atoms beyond ``namespace(pod, ns)``);
* K6 with ``check_select_by_no_policy`` a pod selected by no policy receives
  from and sends to every pod, so edge(src, dst) holds for every pair
  (constraint.py:207-212,222-227,229-231);
* K7 ``policyTypes`` and ports are not used by the relations; a pod in a
  namespace missing from the namespace list raises ``KeyError``
  (constraint.py:251).

Two behaviours of kubesv's encoding are NOT reproduced (intentional
departures, both z3 sort/name artefacts rather than readings of the rules):

* K8 a ``namespaceSelector`` In / NotIn requirement: kubesv declares the
  membership relation over ``pod_sort`` and applies it to a namespace
  variable (model.py:211-221); z3 then raises a sort mismatch whenever the
  pod and namespace bit-vector widths differ, and otherwise ranges over
  namespace ids read as pod ids.  Here the requirement is evaluated on the
  namespace's labels (the Kubernetes meaning).
* K9 namespace label relations are declared as ``Function(k, nam_sort,
  ...)`` under the pod relation's name ``k`` (constraint.py:270, not
  ``k__namespace``); when the two sort widths match that is the same z3
  function as the pod label relation ``k``, so pod and namespace facts on a
  shared key mix.  Here the namespace's labels and the pods' labels stay
  separate columns.

Parity: against ``oracle/kano_oracle.py kubesv_edge_py``, a restatement of
the Datalog rules on Python sets -- unpinned against kubesv itself (it needs
z3 and the kubernetes client, both absent here).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np

from .model import (ReachabilityMatrix, Container, Policy, PolicySelect, PolicyAllow,
                    PolicyEgress, In, NotIn, Exists, DoesNotExist, LabelExpression)

_NS = ("__k8s_namespace__",)


class Namespace:
    """NamespaceAdapter (kubesv/kubesv/model.py:24-50)."""

    def __init__(self, name: str, labels: Optional[Dict[str, Any]] = None):
        self.name = name
        self.labels = dict(labels) if labels else {}


class Pod:
    """PodAdapter (model.py:52-84): namespace defaults to "default"."""

    def __init__(self, name: str, namespace: Optional[str] = None,
                 labels: Optional[Dict[str, Any]] = None):
        self.name = name
        self.namespace = namespace if namespace is not None else "default"
        self.labels = dict(labels) if labels else {}


class NetworkPolicy:
    """PolicyAdapter (model.py:389-553) over a NetworkPolicy spec dict in the
    manifest's camelCase (``podSelector``, ``ingress: [{from: [...]}]``,
    ``egress: [{to: [...]}]``, peers with ``podSelector`` /
    ``namespaceSelector`` / ``ipBlock``, selectors with ``matchLabels`` /
    ``matchExpressions``)."""

    def __init__(self, name: str, namespace: Optional[str] = None,
                 spec: Optional[Dict[str, Any]] = None):
        self.name = name
        self.namespace = namespace if namespace is not None else "default"
        self.spec = spec

    @staticmethod
    def from_manifest(obj: Dict[str, Any]) -> "NetworkPolicy":
        md = obj.get("metadata") or {}
        return NetworkPolicy(md.get("name"), md.get("namespace"), obj.get("spec"))


def from_dict(kind: str, data: Dict[str, Any]):
    """kubesv.parser.from_dict (kubesv/kubesv/parser.py:9-18) without the
    kubernetes client: a manifest dict as this module's Pod / Namespace /
    NetworkPolicy (kind 'V1Pod', 'V1Namespace', 'V1NetworkPolicy'; the 'V1'
    prefix is optional)."""
    k = kind[2:] if kind.startswith("V1") else kind
    md = (data or {}).get("metadata") or {}
    if k == "Pod":
        return Pod(md.get("name"), md.get("namespace"), md.get("labels"))
    if k == "Namespace":
        return Namespace(md.get("name"), md.get("labels"))
    if k == "NetworkPolicy":
        return NetworkPolicy.from_manifest(data)
    raise ValueError(f"unsupported kind {kind!r}")


def from_yaml(kind: str, yml: str):
    """kubesv.parser.from_yaml (parser.py:21-22)."""
    import yaml
    return from_dict(kind, yaml.safe_load(yml))


# ---------------------------------------------------------------------------
# selectors -> requirement terms
# ---------------------------------------------------------------------------

_OPS = {"in": In, "notin": NotIn, "exists": Exists, "doesnotexists": DoesNotExist}


def _terms(selector: Optional[Dict[str, Any]], known: set) -> Optional[List[tuple]]:
    """LabelSelectorAdapter.define_label_selector (model.py:178-233): the
    (key, requirement) terms of a selector, or None on a quick fail (K2)."""
    if selector is None:
        return []
    out = []
    exprs = selector.get("matchExpressions")
    if exprs is not None:
        for e in exprs:
            op = _OPS.get(str(e.get("operator", "")).lower())
            if op is None:
                continue                                  # K3
            if e.get("key") not in known:
                return None                               # K2
            if op in (In, NotIn):
                out.append((e["key"], op(e.get("values") or [])))
            else:
                out.append((e["key"], op()))
    labels = selector.get("matchLabels")
    if labels is not None:
        for k, v in labels.items():
            if k not in known:
                return None                               # K2
            # a plain kano value: key present and equal (Python ==), one
            # shared value column per key rather than a requirement column
            # per term; kano's quirk Q1 cannot fire, some pod carries the key
            out.append((k, v))
    return out


class _TermDict:
    """Terms of one kano selector dict: a key may carry several requirements
    (matchLabels and matchExpressions on one key, or the pod side and the
    namespace side), so repeats go to alias columns holding the same values."""

    def __init__(self, aliases: Dict[Any, Any]):
        self.d: Dict[Any, Any] = {}
        self.aliases = aliases

    def add(self, col, req) -> None:
        key, t = col, 0
        while key in self.d:
            t += 1
            key = ("__alias__", col, t)
            self.aliases[key] = col
        self.d[key] = req


class K8sReachability:
    """kubesv's relations over one cluster, resident on the device."""

    def __init__(self, edge, ingress_traffic, egress_traffic, selected_by_any, info):
        #: edge[src, dst] (constraint.py:229-231), a ReachabilityMatrix
        self.edge = edge
        #: ingress_traffic as [sel, src] and egress_traffic as [sel, dst]
        #: (constraint.py:191-227; the product's two operands)
        self.ingress_traffic = ingress_traffic
        self.egress_traffic = egress_traffic
        #: selected_by_any per pod (constraint.py:179-182), None unless
        #: check_select_by_no_policy asked for it
        self.selected_by_any = selected_by_any
        self.info = info

    def path(self, mode: str = "auto") -> ReachabilityMatrix:
        """path :- edge | edge . edge (constraint.py:233-237)."""
        from .algorithm import two_hop
        return two_hop(self.edge, mode=mode)


def _wrap(engine, n: int) -> ReachabilityMatrix:
    m = ReachabilityMatrix.__new__(ReachabilityMatrix)
    m.container_size = n
    m._engine = engine
    m._containers = None
    m._policies = None
    m._ncontainers = n
    m._lists = None
    return m


def compile_policies(pods: List[Pod], policies: List[NetworkPolicy],
                     namespaces: List[Namespace]):
    """kubesv's facts (constraint.py:242-282) as kano objects: the pods as
    Containers (own labels, namespace, namespace labels, alias columns) and
    three kano policy lists -- ingress peers, egress peers (select = the
    policy's pod selector and namespace, allow = the peer; egress direction,
    so that M[sel][peer pod]) and the bare pod selectors."""
    nam_map = {ns.name: i for i, ns in enumerate(namespaces)}
    by_name = {ns.name: ns for ns in namespaces}
    # define_pod_facts (constraint.py:242-275): the label keys any pod / any
    # namespace carries are the relations a selector may name
    pod_keys, ns_keys = set(), set()
    for p in pods:
        if p.namespace not in nam_map:
            raise KeyError(p.namespace)                  # K7
        pod_keys.update(p.labels.keys())
    for ns in namespaces:
        ns_keys.update(ns.labels.keys())
    # namespace label keys some pod sees (through its namespace)
    ns_pod_keys = set()
    for name in {p.namespace for p in pods}:
        ns_pod_keys.update(by_name[name].labels.keys())

    aliases: Dict[Any, Any] = {}
    ing, egr, sel_only = [], [], []
    for pol in policies:
        spec = pol.spec
        if spec is None:
            raise AttributeError("'NoneType' object has no attribute 'egress'")
        # define_pod_selector (model.py:496-514)
        sel = None
        if pol.namespace in nam_map:
            t = _terms(spec.get("podSelector"), pod_keys)
            if t is not None:
                sel = _TermDict(aliases)
                sel.add(_NS, pol.namespace)
                for k, r in t:
                    sel.add(k, r)
        # define_egress_rules, then define_ingress_rules (constraint.py:278-282)
        for direction, out in (("egress", egr), ("ingress", ing)):
            rules = spec.get(direction)
            if direction == "ingress" and spec.get("egress") is None:
                continue                                  # K4
            if rules is None:
                if direction == "ingress":
                    raise TypeError("'NoneType' object is not iterable")   # K4
                continue
            for rule in rules:
                peers = (rule or {}).get("to" if direction == "egress" else "from")
                if peers is None:
                    raise TypeError("'NoneType' object is not iterable")   # K4
                for peer in peers:
                    peer = peer or {}
                    nst = _terms(peer.get("namespaceSelector"), ns_keys)
                    if nst is None:
                        continue                          # K2
                    pt = _terms(peer.get("podSelector"), pod_keys)
                    if pt is None:
                        continue                          # K2
                    if sel is None:
                        continue                          # selects nothing
                    if any(not isinstance(r, LabelExpression) and k not in ns_pod_keys
                           for k, r in nst):
                        continue      # no pod lives in a namespace with the key
                    alw = _TermDict(aliases)
                    for k, r in nst:
                        alw.add(("__k8s_ns_label__", k), r)
                    for k, r in pt:
                        alw.add(k, r)
                    out.append((sel.d, alw.d))
        if sel is not None:
            sel_only.append((sel.d, {}))

    containers = []
    for p in pods:
        lab = dict(p.labels)
        lab[_NS] = p.namespace
        for k, v in by_name[p.namespace].labels.items():
            lab[("__k8s_ns_label__", k)] = v
        for a, col in aliases.items():
            if col in lab:
                lab[a] = lab[col]
        containers.append(Container(p.name, lab))

    def kano(pairs):
        return [Policy(f"k8s{q}", PolicySelect(s), PolicyAllow(a), PolicyEgress, None)
                for q, (s, a) in enumerate(pairs)]
    return containers, kano(ing), kano(egr), kano(sel_only)


def build(pods: List[Pod], policies: List[NetworkPolicy], namespaces: List[Namespace],
          check_self_ingress_traffic: bool = True, check_select_by_no_policy: bool = False,
          device: int = 0, path: str = "auto", form: str = "classes",
          rows: Optional[tuple] = None, self_term: str = "auto") -> K8sReachability:
    """kubesv's ``build`` (constraint.py:285-299) on the device: the edge
    relation as an n x n matrix (rows src, columns dst).  ``form``: the
    product over the builds' row / column classes ("classes") or over pods
    ("pods"); both give the same matrix.  ``rows=(r0, r1)``: only those rows
    of the edge matrix (a multi-GPU rank's shard; the class form).
    ``self_term``: "expand" (from the egress classes), "build" (the
    destination is a build of the egress policies) or "auto"."""
    from ._engine import DeviceBuild
    from ._intern import intern
    containers, ing, egr, sel_only = compile_policies(pods, policies, namespaces)
    n = len(pods)

    def operand(pols):
        b = DeviceBuild(intern(containers, pols), device=device, path=path, build=False)
        b.build_classes(path)          # Mc and classes; M written only if read
        return b

    in_t = operand(ing)
    eg_t = operand(egr)
    selected = None
    all_pairs = False
    if check_select_by_no_policy:
        # a pod is selected by some policy iff its row class's S(c) is not
        # empty: the class-level build only (no matrix is written or
        # allocated, whatever n and rows are)
        selected = np.zeros(n, dtype=bool)
        if n:
            ms = DeviceBuild(intern(containers, sel_only), device=device, path=path,
                             build=False)
            ms.build_classes(path)
            off, _ = ms.select_csr()
            selected = np.diff(off)[ms.classes()] > 0
            ms.close()
        all_pairs = bool(n) and not bool(selected.all())
    # the self term: expanded from the egress classes ("expand", the
    # default), or the destination is a build of the egress policies over its
    # rows, whose matrix write is the term ("build"; measured 0.89 vs 2.4 ms
    # at 100k pods, and 26-29 vs 22-428 ms for 1M pods' rank 0 of 8, where
    # the destination's 15.6 GB allocation inside the call varies widely)
    big = self_term == "build"
    in_place = (bool(check_self_ingress_traffic) and not all_pairs and form == "classes"
                and n > 0 and big)
    if in_place:
        # the destination is a build of the egress policies over its rows:
        # its matrix write is the self term (EgT's rows), the product is
        # OR-ed into it
        out = DeviceBuild(eg_t.tables, device=device, rows=rows, path=path)
    else:
        out = DeviceBuild.empty(n, device=device, rows=rows)
    added = out.k8s_edge_from(in_t, eg_t, bool(check_self_ingress_traffic), all_pairs,
                              pods=(form == "pods"), dst_is_egress=in_place)
    info = {"ingress_policies": len(ing), "egress_policies": len(egr),
            "product_bits": added, "all_pairs": all_pairs, "rows": rows}
    return K8sReachability(_wrap(out, n), _wrap(in_t, n), _wrap(eg_t, n), selected, info)
