"""Incremental policy updates: after
ReachabilityMatrix.add_policies / remove_policies the matrix, the containers'
select_policies / allow_policies, the policies' working sets and every check
equal a fresh build_matrix over the updated policy list (kano_py/kano/
model.py:125-165), bit for bit.  The fresh builds are pinned to kano_py by
tests/test_gpu_parity.py."""
import copy

import numpy as np
import pytest

from _golden import cluster

pytestmark = pytest.mark.gpu


def _objs(obj):
    from kano import model
    from kano.synth import objects_from_json
    return objects_from_json(obj, model)


def _state(m, cs, ps):
    from kano import algorithm as alg
    n = m.container_size
    out = {"M": m.engine.rows(0, n),
           "sel": [list(c.select_policies) for c in cs],
           "alw": [list(c.allow_policies) for c in cs],
           "wsel": [p.working_select_set.tolist() for p in ps],
           "walw": [p.working_allow_set.tolist() for p in ps],
           "reach": alg.all_reachable(m), "iso": alg.all_isolated(m),
           "cross": alg.user_crosscheck(m, cs, "tenant" if any(
               "tenant" in c.labels for c in cs) else "app"),
           "sys": alg.system_isolation(m, 0) if n else [],
           "shadow": alg.policy_shadow(m, ps, cs)}
    try:
        out["conflict"] = alg.policy_conflict(m, ps, cs)
    except AttributeError as e:
        out["conflict"] = str(e)
    return out


def _fresh(obj, keep):
    from kano.model import ReachabilityMatrix
    cs, ps = _objs(obj)
    ps = [ps[k] for k in keep]
    m = ReachabilityMatrix.build_matrix(cs, ps)
    return _state(m, cs, ps)


def _assert_same(a, b):
    assert np.array_equal(a["M"], b["M"])
    for k in ("sel", "alw", "wsel", "walw", "reach", "iso", "cross", "sys", "shadow", "conflict"):
        assert a[k] == b[k], k


@pytest.mark.parametrize("name", ["q_dirs", "q_shadow", "s_sparse_200", "s_sparse_1000",
                                  "s_broad_300"])
def test_add_equals_rebuild(name):
    from kano.model import ReachabilityMatrix
    obj = cluster(name)
    cs, ps = _objs(obj)
    P = len(ps)
    k = max(1, P // 5)
    base, extra = ps[:P - k], ps[P - k:]
    m = ReachabilityMatrix.build_matrix(cs, base)
    m.add_policies(extra[:1])
    m.add_policies(extra[1:])
    assert base is m._policies and len(base) == P
    _assert_same(_state(m, cs, base), _fresh(obj, range(P)))


@pytest.mark.parametrize("name", ["q_dirs", "s_sparse_200", "s_sparse_1000", "s_broad_300"])
def test_remove_equals_rebuild(name):
    from kano.model import ReachabilityMatrix
    obj = cluster(name)
    cs, ps = _objs(obj)
    P = len(ps)
    gone = sorted({0, P // 3, P // 2, P - 1})
    m = ReachabilityMatrix.build_matrix(cs, ps)
    m.remove_policies(gone)
    keep = [p for p in range(P) if p not in gone]
    _assert_same(_state(m, cs, ps), _fresh(obj, keep))


def test_mixed_sequence_with_new_keys_and_matchers():
    """add (one policy on a key no earlier policy used, one with a custom
    matcher), remove a build policy and an added one, add again."""
    from kano import model
    from kano.model import ReachabilityMatrix
    obj = copy.deepcopy(cluster("s_sparse_500"))
    cs, ps = _objs(obj)
    P = len(ps)

    class Prefix(model.DefaultEqualityLabelRelation):
        def match(self, rule, value):
            return isinstance(value, str) and value.startswith(rule)

    def extra_policies():
        keys = sorted({k for c in cs for k in c.labels})
        used = {k for p in ps for k in list(p.selector.labels) + list(p.allow.labels)}
        fresh = [k for k in keys if k not in used] or keys
        c0 = cs[3]
        k0 = fresh[0]
        v0 = next(c.labels[k0] for c in cs if k0 in c.labels)
        a = model.Policy("x_newkey", model.PolicySelect({k0: v0}),
                         model.PolicyAllow(dict(list(c0.labels.items())[:1])),
                         model.PolicyEgress, model.PolicyProtocol(["TCP"]))
        kk = next(iter(c0.labels))
        b = model.Policy("x_prefix", model.PolicySelect({kk: str(c0.labels[kk])[:2]}),
                         model.PolicyAllow({}), model.PolicyIngress,
                         model.PolicyProtocol(["TCP"]), matcher=Prefix())
        c = model.Policy("x_late", model.PolicySelect({}), model.PolicyAllow({kk: c0.labels[kk]}),
                         model.PolicyEgress, model.PolicyProtocol(["TCP"]))
        return a, b, c

    a, b, c = extra_policies()
    m = ReachabilityMatrix.build_matrix(cs, ps)
    m.add_policies([a, b])                     # ids P, P+1
    m.remove_policies([5, P])                  # a build policy and `a`
    m.add_policies([c])
    got = _state(m, cs, ps)
    # the same list built from scratch (fresh objects)
    cs2, ps2 = _objs(obj)
    a2, b2, c2 = a, b, c
    final = [ps2[k] for k in range(P) if k != 5] + [b2, c2]
    m2 = ReachabilityMatrix.build_matrix(cs2, final)
    _assert_same(got, _state(m2, cs2, final))


def test_remove_after_edit_raises():
    from kano.model import ReachabilityMatrix
    from kano._native import KanoNativeError
    cs, ps = _objs(cluster("s_sparse_50"))
    m = ReachabilityMatrix.build_matrix(cs, ps)
    m[0, 1] = 1
    with pytest.raises(KanoNativeError):
        m.remove_policies([0])


# --- pinned to the oracle (the reference's algorithm over the updated list) --
def _oracle(obj, keep, extra=()):
    """oracle.run_c (the C restatement pinned to kano_py) over the policy
    list [policies[k] for k in keep] + extra: what build_matrix over the
    updated list gives (kano_py/kano/model.py:125-165, algorithm.py:4-80)."""
    from oracle import kano_oracle as orc
    o = dict(obj)
    o["policies"] = [obj["policies"][k] for k in keep] + list(extra)
    return orc.run_c(o, label=obj.get("label", "app"))


def _csr_lists(off, lst):
    return [lst[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]


def _check_vs_oracle(m, cs, ps, ref, label):
    from kano import algorithm as alg
    n = m.container_size
    assert np.array_equal(m.engine.rows(0, n), ref["M"])
    assert [list(c.select_policies) for c in cs] == _csr_lists(ref["select_off"],
                                                                ref["select_list"])
    assert [list(c.allow_policies) for c in cs] == _csr_lists(ref["allow_off"], ref["allow_list"])
    assert alg.all_reachable(m) == ref["all_reachable"]
    assert alg.all_isolated(m) == ref["all_isolated"]
    assert alg.user_crosscheck(m, cs, label) == ref["user_crosscheck"]
    assert alg.system_isolation(m, 0) == ref["system_isolation"]
    assert np.array_equal(np.array(alg.policy_shadow(m, ps, cs), np.int32).reshape(-1, 2),
                          ref["shadow"].reshape(-1, 2))


@pytest.mark.parametrize("name", ["q_dirs", "q_shadow", "s_sparse_200", "s_sparse_1000",
                                  "s_broad_300", "q_wide_select"])
def test_remove_then_add_vs_oracle(name):
    """remove_policies, then add_policies, each against the oracle over the
    updated policy list -- not against another GPU build."""
    from kano import model
    from kano.model import ReachabilityMatrix
    obj = cluster(name)
    label = obj.get("label", "app")
    cs, ps = _objs(obj)
    P = len(ps)
    gone = sorted({0, P // 3, P // 2, P - 1})
    keep = [p for p in range(P) if p not in gone]
    m = ReachabilityMatrix.build_matrix(cs, ps)
    m.remove_policies(gone)
    _check_vs_oracle(m, cs, ps, _oracle(obj, keep), label)
    # add two removed policies back (now at the end of the list)
    back = [obj["policies"][gone[0]], obj["policies"][gone[-1]]]
    m.add_policies([_policy(model, q) for q in back])
    _check_vs_oracle(m, cs, ps, _oracle(obj, keep, back), label)


def _policy(model, q):
    d = model.PolicyIngress if q["direction"] == "ingress" else model.PolicyEgress
    return model.Policy(q["name"], model.PolicySelect(q["select"]), model.PolicyAllow(q["allow"]),
                        d, model.PolicyProtocol(q.get("protocol") or []))


@pytest.mark.parametrize("name", ["q_dirs", "s_sparse_200", "s_broad_300"])
def test_remove_after_second_build_keeps_first_builds_entries(name):
    """Quirk Q5: a second build on the same containers appends after the
    first build's entries; removing a policy from the second matrix
    renumbers only its own entries (the first build's stay as that build
    appended them)."""
    from kano.model import ReachabilityMatrix
    obj = cluster(name)
    cs, ps = _objs(obj)
    ps2 = list(ps)
    P = len(ps)
    ReachabilityMatrix.build_matrix(cs, ps)          # build 1 (over all P)
    m2 = ReachabilityMatrix.build_matrix(cs, ps2)    # build 2 accumulates
    gone = sorted({1, P // 2})
    m2.remove_policies(gone)
    keep = [p for p in range(P) if p not in gone]
    first = _oracle(obj, range(P))
    second = _oracle(obj, keep)
    assert np.array_equal(m2.engine.rows(0, len(cs)), second["M"])
    s1, s2 = (_csr_lists(r["select_off"], r["select_list"]) for r in (first, second))
    a1, a2 = (_csr_lists(r["allow_off"], r["allow_list"]) for r in (first, second))
    assert [list(c.select_policies) for c in cs] == [x + y for x, y in zip(s1, s2)]
    assert [list(c.allow_policies) for c in cs] == [x + y for x, y in zip(a1, a2)]


@pytest.mark.parametrize("name,spans", [
    ("s_sparse_1000", [(0, 300), (300, 301), (301, 1000)]),
    ("s_broad_300", [(0, 150), (150, 300)]),
    ("q_wide_select", [(0, 400), (400, 800), (800, 1200)]),
])
def test_incremental_on_row_shards_recombine(name, spans):
    """add / remove on every rank's row shard (kano_add_policies /
    kano_remove_policies write only the shard's rows), then the checks over
    the rows as they stand (kano_checks_shard) gathered and combined
    (kano_verify_combine): equal to the oracle over the updated list, and
    the shards' rows equal the oracle's matrix."""
    import torch
    from kano import model
    from kano._engine import DeviceBuild
    from kano._intern import group_ids, intern, intern_more
    obj = cluster(name)
    label = obj.get("label", "app")
    cs, ps = _objs(obj)
    P = len(ps)
    t = intern(cs, ps)
    gid = group_ids(cs, label)
    n = t.n
    W = (n + 63) // 64
    gone = [1, P - 2]
    extra = [obj["policies"][3], obj["policies"][P // 2]]
    keep = [p for p in range(P) if p not in gone]
    ref = _oracle(obj, keep, extra)
    N = len(spans)
    gathered = torch.zeros(N * 3 * W, dtype=torch.int64, device="cuda")
    engs = []
    for k, (r0, r1) in enumerate(spans):
        # every rank interns for itself (intern_more extends the interning
        # state of the rank's own tables)
        e = DeviceBuild(intern(cs, ps), rows=(r0, r1))
        e.remove_policies(gone)
        xval, sel, alw = intern_more(e.tables, [_policy(model, q) for q in extra])
        e.add_policies(xval, sel, alw)
        assert np.array_equal(e.rows(r0, r1 - r0), ref["M"][r0:r1]), f"shard {k} rows"
        e.checks_shard(gathered.data_ptr() + 8 * 3 * W * k, gid=gid, sys_row=0)
        engs.append(e)
    torch.cuda.synchronize()
    for k, ((r0, r1), e) in enumerate(zip(spans, engs)):
        r = e.verify_combine(gathered.data_ptr(), N)
        assert r["all_reachable"].tolist() == ref["all_reachable"]
        assert r["all_isolated"].tolist() == ref["all_isolated"]
        assert r["user_crosscheck"].tolist() == ref["user_crosscheck"]
        if r0 <= 0 < r1:
            assert r["system_isolation"].tolist() == ref["system_isolation"]
        else:
            assert r["system_isolation"] is None
        e.close()
