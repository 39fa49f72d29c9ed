"""kubesv's Kubernetes relations on kano's engine:
namespaces, namespaceSelector, per-direction rules, self traffic and pods
selected by no policy (kubesv/kubesv/model.py, constraint.py:168-237).

kubesv needs z3 and the kubernetes client (both absent), so parity is against
the Datalog rules restated on Python sets (oracle/kano_oracle.py
kubesv_edge_py), written independently of kano/k8s.py's compilation to kano
policies: parity unpinned against a kubesv run.  The GPU edge matrix
(libkano_hip.so kano_k8s_edge) must equal the restatement bit for bit."""
import random

import numpy as np
import pytest

NS_LABELS = [{"team": "a", "env": "prod"}, {"team": "b"}, {"env": "dev"}, {}, {"team": "a"}]


def _selector(rnd, keys, vals, allow_none=True):
    if allow_none and rnd.random() < 0.15:
        return None
    s = {}
    if rnd.random() < 0.7:
        s["matchLabels"] = {k: rnd.choice(vals) for k in rnd.sample(keys, rnd.randint(0, 2))}
    if rnd.random() < 0.5:
        ex = []
        for _ in range(rnd.randint(0, 2)):
            op = rnd.choice(["In", "NotIn", "Exists", "DoesNotExist", "doesnotexists", "bogus"])
            e = {"key": rnd.choice(keys), "operator": op}
            if op in ("In", "NotIn"):
                e["values"] = rnd.sample(vals, 2)
            ex.append(e)
        s["matchExpressions"] = ex
    return s


def _cluster(seed, n=60, P=25, nns=4):
    from kano import k8s
    rnd = random.Random(seed)
    nss = [k8s.Namespace(f"ns{i}", NS_LABELS[i % len(NS_LABELS)]) for i in range(nns)]
    pods = []
    for i in range(n):
        lab = {"app": rnd.choice(["web", "db", "cache", "api"])}
        if rnd.random() < 0.6:
            lab["tier"] = rnd.choice(["fe", "be"])
        if rnd.random() < 0.2:
            lab["ver"] = rnd.choice([1, 2, "1"])
        pods.append(k8s.Pod(f"p{i}", rnd.choice([None] + [ns.name for ns in nss]), lab))
    nss.append(k8s.Namespace("default", {"team": "c"}))
    pod_keys = ["app", "tier", "ver", "zone"]             # zone: no pod carries it (K2)
    pod_vals = ["web", "db", "api", "fe", "be", 1, "1"]
    ns_keys = ["team", "env", "region"]                   # region: no namespace carries it
    ns_vals = ["a", "b", "c", "prod", "dev"]

    def narrow(keys, vals):
        if rnd.random() < 0.6:
            return {"matchLabels": {keys[0]: rnd.choice(vals)}}
        return _selector(rnd, keys, vals, allow_none=False)

    def peer():
        r = rnd.random()
        if r < 0.02:
            return {"ipBlock": {"cidr": "10.0.0.0/8"}}    # K5
        p = {}
        if r < 0.75:
            p["podSelector"] = narrow(pod_keys, pod_vals)
        if r > 0.5:
            p["namespaceSelector"] = narrow(ns_keys, ns_vals)
        return p

    def rules(key):
        return [{key: [peer() for _ in range(rnd.randint(0, 2))]}
                for _ in range(rnd.randint(0, 2))]

    pols = []
    for q in range(P):
        spec = {"podSelector": (narrow(pod_keys, pod_vals) if rnd.random() < 0.9
                                else _selector(rnd, pod_keys, pod_vals))}
        r = rnd.random()
        if r < 0.75:
            spec["egress"] = rules("to")
            spec["ingress"] = rules("from")
        elif r < 0.9:
            spec["ingress"] = rules("from")               # K4: ignored without egress
        ns = rnd.choice([ns.name for ns in nss] + [None, "ghost"])
        pols.append(k8s.NetworkPolicy(f"np{q}", ns, spec))
    return pods, pols, nss


def _bits(M, n):
    return {(i, j) for i in range(n) for j in range(n) if (int(M[i, j >> 6]) >> (j & 63)) & 1}


def test_oracle_small_cases():
    """The restated rules on hand-checked cases (constraint.py:191-231)."""
    from kano import k8s
    from oracle import kano_oracle as orc
    nss = [k8s.Namespace("a", {"team": "x"}), k8s.Namespace("b", {})]
    pods = [k8s.Pod("w", "a", {"app": "web"}), k8s.Pod("d", "a", {"app": "db"}),
            k8s.Pod("o", "b", {"app": "web"})]
    # db accepts ingress from web pods of team-x namespaces; sends to anyone
    pol = k8s.NetworkPolicy("p", "a", {
        "podSelector": {"matchLabels": {"app": "db"}},
        "ingress": [{"from": [{"podSelector": {"matchLabels": {"app": "web"}},
                               "namespaceSelector": {"matchLabels": {"team": "x"}}}]}],
        "egress": [{"to": [{}]}]})
    edge, ing, eg = orc.kubesv_edge_py(pods, [pol], nss, check_self_ingress_traffic=False)
    assert ing[1] == {0} and eg[1] == {0, 1, 2}
    assert edge == {(0, 0), (0, 1), (0, 2)}
    edge, _, _ = orc.kubesv_edge_py(pods, [pol], nss)       # + self: d -> egress of d
    assert edge == {(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2)}
    # K4: without egress the ingress rules are not defined
    pol2 = k8s.NetworkPolicy("p", "a", {"podSelector": {}, "ingress": pol.spec["ingress"]})
    edge, ing, _ = orc.kubesv_edge_py(pods, [pol2], nss, check_self_ingress_traffic=False)
    assert edge == set() and all(not v for v in ing.values())
    # K6: a pod selected by no policy makes every pair an edge
    edge, _, _ = orc.kubesv_edge_py(pods, [pol], nss, check_select_by_no_policy=True)
    assert len(edge) == 9


def test_host_errors_match_kubesv():
    """K4 / K7: kubesv's TypeError and KeyError, raised before any device work."""
    from kano import k8s
    nss = [k8s.Namespace("default")]
    pods = [k8s.Pod("a", None, {"x": "1"})]
    with pytest.raises(TypeError):
        k8s.build(pods, [k8s.NetworkPolicy("p", None, {"egress": [], "ingress": None})], nss)
    with pytest.raises(TypeError):
        k8s.build(pods, [k8s.NetworkPolicy("p", None, {"egress": [{"to": None}]})], nss)
    with pytest.raises(KeyError):
        k8s.build([k8s.Pod("a", "nowhere")], [], nss)


def test_compiled_terms_cover_quirks():
    """The selector compilation (kano/k8s.py _terms): K2 quick fail, K3
    operator spelling, requirement objects for every term."""
    from kano import k8s
    from kano.model import In, NotIn, Exists, DoesNotExist
    known = {"app", "tier"}
    assert k8s._terms(None, known) == []
    assert k8s._terms({"matchLabels": {"zone": "x"}}, known) is None
    t = k8s._terms({"matchExpressions": [
        {"key": "app", "operator": "In", "values": ["a"]},
        {"key": "tier", "operator": "DoesNotExist"},          # dropped (K3)
        {"key": "tier", "operator": "doesnotexists"},
        {"key": "app", "operator": "NotIn", "values": ["b"]},
        {"key": "tier", "operator": "Exists"}], "matchLabels": {"app": "web"}}, known)
    assert [(k, type(r)) for k, r in t] == [("app", In), ("tier", DoesNotExist),
                                           ("app", NotIn), ("tier", Exists), ("app", str)]


def _ref_rows(cs, ps, n):
    from oracle import kano_oracle as orc
    if n == 0:
        return np.zeros((0, 0), bool)
    M = orc.ref_py(cs, ps)["M"]
    return np.array([[c == "1" for c in r] for r in M], dtype=bool).reshape(n, n)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("self_traffic", [True, False])
def test_compilation_matches_oracle(seed, self_traffic):
    """kano/k8s.py's compilation to kano policies, evaluated by the kano
    restatement (oracle ref_py) and multiplied in numpy, equals the kubesv
    rules restated on sets: the device only has to compute the kano matrices
    and the product right."""
    from kano import k8s
    from oracle import kano_oracle as orc
    pods, pols, nss = _cluster(seed, n=40, P=20)
    n = len(pods)
    cs, ing, egr, _ = k8s.compile_policies(pods, pols, nss)
    InT = _ref_rows(cs, ing, n)
    EgT = _ref_rows(cs, egr, n)
    E = (InT.T.astype(np.int64) @ EgT.astype(np.int64)) > 0
    if self_traffic:
        E |= EgT
    edge, ing_s, eg_s = orc.kubesv_edge_py(pods, pols, nss, self_traffic, False)
    assert {(int(i), int(j)) for i, j in zip(*np.nonzero(E))} == edge
    _, ing0, eg0 = orc.kubesv_edge_py(pods, pols, nss, False, False)
    assert {(int(i), int(j)) for i, j in zip(*np.nonzero(InT))} == {
        (s, x) for s in range(n) for x in ing0[s]}
    assert {(int(i), int(j)) for i, j in zip(*np.nonzero(EgT))} == {
        (s, x) for s in range(n) for x in eg0[s]}


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("self_traffic,by_none", [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize("form", ["classes", "pods", "classes+build"])
def test_edge_matches_oracle(seed, self_traffic, by_none, form):
    from kano import k8s
    from oracle import kano_oracle as orc
    pods, pols, nss = _cluster(seed)
    n = len(pods)
    r = k8s.build(pods, pols, nss, check_self_ingress_traffic=self_traffic,
                  check_select_by_no_policy=by_none, form=form.split("+")[0],
                  self_term="build" if form.endswith("build") else "expand")
    edge, ing, eg = orc.kubesv_edge_py(pods, pols, nss, self_traffic, by_none)
    assert _bits(r.edge.engine.rows(0, n), n) == edge
    # the product's operands: ingress_traffic [sel][src] without the self
    # term (added in the product), egress_traffic [sel][dst]
    _, ing0, eg0 = orc.kubesv_edge_py(pods, pols, nss, False, False)
    assert _bits(r.ingress_traffic.engine.rows(0, n), n) == {
        (s, x) for s in range(n) for x in ing0[s]}
    assert _bits(r.egress_traffic.engine.rows(0, n), n) == {
        (s, x) for s in range(n) for x in eg0[s]}
    if by_none:
        unsel = [s for s in range(n) if len(eg[s]) == n and len(ing[s]) == n]
        assert r.info["all_pairs"] == (len(edge) == n * n and bool(unsel))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 7, 0])
def test_edge_checks_and_path(seed):
    """Every kano check and kubesv's path relation read the edge matrix."""
    from kano import algorithm as alg, k8s
    from oracle import kano_oracle as orc
    pods, pols, nss = _cluster(seed, n=90, P=30)
    n = len(pods)
    r = k8s.build(pods, pols, nss)
    edge, _, _ = orc.kubesv_edge_py(pods, pols, nss)
    assert alg.all_isolated(r.edge) == [j for j in range(n)
                                        if not any((i, j) in edge for i in range(n))]
    assert alg.all_reachable(r.edge) == [j for j in range(n)
                                         if all((i, j) in edge for i in range(n))]
    assert alg.system_isolation(r.edge, 0) == [j for j in range(n) if (0, j) not in edge]
    p = r.path()
    assert _bits(p.engine.rows(0, n), n) == orc.path_py(edge, n, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["classes", "pods"])
@pytest.mark.parametrize("seed,self_traffic", [(99, True), (5, False)])
def test_edge_larger_cluster(form, seed, self_traffic):
    """A few thousand pods: many words per row, both product forms."""
    from kano import k8s
    from oracle import kano_oracle as orc
    pods, pols, nss = _cluster(seed, n=1500, P=20, nns=5)
    n = len(pods)
    r = k8s.build(pods, pols, nss, check_self_ingress_traffic=self_traffic, form=form)
    edge, _, _ = orc.kubesv_edge_py(pods, pols, nss, self_traffic)
    M = r.edge.engine.rows(0, n)
    ref = np.zeros_like(M)
    for i, j in edge:
        ref[i, j >> 6] |= np.uint64(1) << np.uint64(j & 63)
    assert np.array_equal(M, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("cuts", [[0, 30, 60], [0, 1, 59, 60], [0, 20, 20, 45, 60]])
@pytest.mark.parametrize("self_traffic", [True, False])
@pytest.mark.parametrize("self_term", ["expand", "build"])
def test_edge_row_shards(cuts, self_traffic, self_term):
    """A rank's rows of the edge matrix (rows=(r0, r1)), recombined, equal
    the whole matrix and the restated rules (the multi-GPU split)."""
    from kano import k8s
    from oracle import kano_oracle as orc
    pods, pols, nss = _cluster(5)
    n = len(pods)
    edge, _, _ = orc.kubesv_edge_py(pods, pols, nss, self_traffic)
    parts = []
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        r = k8s.build(pods, pols, nss, check_self_ingress_traffic=self_traffic, rows=(r0, r1),
                      self_term=self_term)
        parts.append(r.edge.engine.rows(r0, r1 - r0))
    M = np.concatenate(parts, axis=0)
    assert M.shape[0] == n
    assert _bits(M, n) == edge


@pytest.mark.gpu
def test_edge_row_shard_checks_refuse_and_by_none():
    """A row shard's edge is not a whole matrix: kano.algorithm's column
    checks refuse it (they would fold only the rank's rows) instead of
    answering for the shard; with check_select_by_no_policy the shards,
    recombined, still equal the restated rules."""
    from kano import k8s, algorithm
    from oracle import kano_oracle as orc
    pods, pols, nss = _cluster(5)
    n = len(pods)
    r = k8s.build(pods, pols, nss, rows=(20, 45))
    with pytest.raises(ValueError):
        algorithm.all_isolated(r.edge)
    with pytest.raises(ValueError):
        algorithm.all_reachable(r.edge)
    edge, _, _ = orc.kubesv_edge_py(pods, pols, nss, True, True)
    parts = []
    for r0, r1 in [(0, 25), (25, n)]:
        rr = k8s.build(pods, pols, nss, rows=(r0, r1), check_select_by_no_policy=True)
        parts.append(rr.edge.engine.rows(r0, r1 - r0))
    assert _bits(np.concatenate(parts, axis=0), n) == edge


@pytest.mark.gpu
def test_build_classes_defers_the_matrix():
    """kano_build_classes: the same classes and checks as kano_build, and the
    same matrix once it is read (written on first use)."""
    from kano import model
    from kano._engine import DeviceBuild
    from kano._intern import intern
    from kano.synth import make_cluster, cluster_objects
    cs, ps = cluster_objects(make_cluster(800, 80, seed=4), model)
    t = intern(cs, ps)
    a = DeviceBuild(t)
    b = DeviceBuild(t, build=False)
    b.build_classes()
    ia, ib = a.info(), b.info()
    # (ROWS_KERNEL / ROWS_CUS name the matrix write that ran: none yet in b)
    assert ia.pop("ROWS_KERNEL") == 2 and ib.pop("ROWS_KERNEL") == 0
    assert ia.pop("ROWS_CUS") > 0 and ib.pop("ROWS_CUS") == 0
    assert ia == ib
    assert np.array_equal(a.rows(0, 800), b.rows(0, 800))


# kubesv's sample cluster (kubesv/sample/example.py:106-174; its test,
# kubesv/tests/test_basic.py:13-30, queries egress_traffic with self ingress
# traffic on).  Worked by hand from the rules: the policy selects the two db
# pods of "default" (0, 1); egress goes to tomcat pods of namespaces without
# "l" (8, 9); ingress comes from tomcat pods of nonsense=default namespaces
# (8, 9) and, with self traffic, from the selected pod itself.
PAPER_EGRESS = {(8, 0), (9, 0), (8, 1), (9, 1)}                   # (dst, sel)
PAPER_EDGE = {(s, d) for s in (0, 1, 8, 9) for d in (8, 9)}            # (src, dst)


def test_paper_example_oracle():
    from sample.kubesv_example import paper_example
    from oracle import kano_oracle as orc
    pods, pols, nss = paper_example()
    assert [p.name for p in pods][:2] == ["db_0", "db_1"] and pols[0].namespace == "default"
    edge, ing, eg = orc.kubesv_edge_py(pods, pols, nss, True, False)
    assert {(d, s) for s in range(len(pods)) for d in eg[s]} == PAPER_EGRESS
    assert edge == PAPER_EDGE


@pytest.mark.gpu
@pytest.mark.parametrize("self_term", ["expand", "build"])
def test_paper_example_gpu(self_term):
    from kano import k8s, algorithm as alg
    from sample.kubesv_example import paper_example
    pods, pols, nss = paper_example()
    n = len(pods)
    r = k8s.build(pods, pols, nss, check_self_ingress_traffic=True,
                  check_select_by_no_policy=False, self_term=self_term)
    assert {(d, s) for s, d in _bits(r.egress_traffic.engine.rows(0, n), n)} == PAPER_EGRESS
    assert _bits(r.edge.engine.rows(0, n), n) == PAPER_EDGE
    assert alg.all_isolated(r.edge) == [j for j in range(n) if j not in (8, 9)]


def test_from_yaml_manifests():
    """kano.k8s.from_yaml reads the manifests kubesv's parser deserialises
    (kubesv/kubesv/parser.py:9-22): metadata name / namespace / labels, the
    NetworkPolicy spec as written."""
    from kano import k8s
    pod = k8s.from_yaml("V1Pod", """
apiVersion: v1
kind: Pod
metadata: {name: label-demo, labels: {environment: production, app: nginx}}
spec: {containers: [{name: nginx, image: "nginx:1.14.2"}]}
""")
    assert (pod.name, pod.namespace, pod.labels) == (
        "label-demo", "default", {"environment": "production", "app": "nginx"})
    ns = k8s.from_yaml("Namespace", "kind: Namespace\nmetadata: {name: shop, labels: {team: a}}\n")
    assert (ns.name, ns.labels) == ("shop", {"team": "a"})
    pol = k8s.from_yaml("V1NetworkPolicy", """
kind: NetworkPolicy
metadata: {name: default-deny-all, namespace: default}
spec: {podSelector: {}, ingress: []}
""")
    assert pol.namespace == "default" and pol.spec == {"podSelector": {}, "ingress": []}
    with pytest.raises(ValueError):
        k8s.from_dict("V1Service", {})
