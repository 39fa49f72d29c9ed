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
