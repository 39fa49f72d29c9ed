"""matchExpressions requirements (an extension of
kano_py's equality selectors): In / NotIn / Exists / DoesNotExist values in
PolicySelect / PolicyAllow, evaluated on the device (kano_set_expressions,
k_expr_cols) and joined like any other term.  Semantics: the label-selector
requirements kubesv adapts (kubesv/kubesv/model.py:127-160).  kubesv needs z3
and the kubernetes client (absent), so parity is against the restated
semantics in oracle/kano_oracle.py ref_py: parity unpinned against a
reference run."""
import random

import numpy as np
import pytest


def _cluster(seed, n=120, P=40):
    from kano import model
    rnd = random.Random(seed)
    apps = ["web", "db", "cache", "api", 7, 7.0]
    cs = []
    for i in range(n):
        lab = {"app": rnd.choice(apps)}
        if rnd.random() < 0.6:
            lab["tier"] = rnd.choice(["fe", "be"])
        if rnd.random() < 0.3:
            lab["env"] = rnd.choice(["prod", "dev", float("nan")])
        cs.append(model.Container(f"c{i}", lab))

    def side():
        d = {}
        for _ in range(rnd.randint(0, 3)):
            k = rnd.choice(["app", "tier", "env", "zone"])      # zone: no pod has it
            r = rnd.random()
            if r < 0.2:
                d[k] = model.In(rnd.sample(["web", "db", "fe", "prod", 7, "x"], 2))
            elif r < 0.4:
                d[k] = model.NotIn(rnd.sample(["web", "db", "be", "dev", 7], 2))
            elif r < 0.5:
                d[k] = model.Exists()
            elif r < 0.6:
                d[k] = model.DoesNotExist()
            else:
                d[k] = rnd.choice(["web", "db", "fe", "be", "prod", 7])
        return d

    ps = [model.Policy(f"p{p}", model.PolicySelect(side()), model.PolicyAllow(side()),
                       rnd.choice([model.PolicyIngress, model.PolicyEgress]),
                       model.PolicyProtocol(["TCP"])) for p in range(P)]
    return cs, ps


def test_host_predicate_matches_oracle():
    """Policy.select_policy / allow_policy (model.py:95-111 plus requirements)
    agree with the oracle's restatement on every container."""
    from oracle import kano_oracle as orc
    for seed in range(5):
        cs, ps = _cluster(seed)
        ref = orc.ref_py(cs, ps)
        keys = {k for c in cs for k in c.labels}
        for p, pol in enumerate(ps):
            for i, c in enumerate(cs):
                pres = all(k in c.labels for k, r in pol.working_selector.labels.items()
                           if k in keys and not hasattr(r, "matches"))
                assert int(pres and pol.select_policy(c)) == int(ref["sel"][p][i])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_expressions_match_oracle(seed):
    from kano import algorithm as alg
    from kano.model import ReachabilityMatrix
    from oracle import kano_oracle as orc
    cs, ps = _cluster(seed)
    ref = orc.ref_py(cs, ps)
    m = ReachabilityMatrix.build_matrix(cs, ps)
    n = m.container_size
    from _golden import words_to_rows01
    assert words_to_rows01(m.engine.rows(0, n), n) == ref["M"]
    assert ["".join(str(int(b)) for b in p.working_select_set.tolist()) for p in ps] == ref["sel"]
    assert ["".join(str(int(b)) for b in p.working_allow_set.tolist()) for p in ps] == ref["allow"]
    assert [list(c.select_policies) for c in cs] == ref["select_policies"]
    assert alg.all_isolated(m) == ref["all_isolated"]
    assert alg.policy_shadow(m, ps, cs) == ref["policy_shadow"]


@pytest.mark.gpu
def test_expressions_incremental():
    """An added policy with requirements (host-evaluated extra columns)
    equals a build over the full list."""
    from kano.model import ReachabilityMatrix
    cs, ps = _cluster(11)
    cs2, ps2 = _cluster(11)
    m = ReachabilityMatrix.build_matrix(cs, ps[:30])
    m.add_policies(ps[30:])
    m2 = ReachabilityMatrix.build_matrix(cs2, ps2)
    n = len(cs)
    assert np.array_equal(m.engine.rows(0, n), m2.engine.rows(0, n))
    assert [c.select_policies for c in cs] == [c.select_policies for c in cs2]
