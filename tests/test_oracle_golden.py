"""The oracle pinned against kano_py's own outputs (tests/golden/expected,
produced by running the reference, tests/golden/make_golden.py).  CPU only."""
import os
import sys

import numpy as np
import pytest

from _golden import (GOLDEN, cluster, cluster_names, csr_sha, expected, lists_to_csr,
                     rows01_to_words, sha, words_to_rows01)
from oracle import kano_oracle as orc

sys.path.insert(0, GOLDEN)


def paper_json():
    from sample import paper_example
    cs, ps = paper_example()
    return {
        "pods": [{"name": c.name, "labels": c.labels} for c in cs],
        "policies": [{"name": p.name, "select": p.selector.labels, "allow": p.allow.labels,
                      "direction": "ingress" if p.is_ingress() else "egress"} for p in ps],
    }


def check_record(res, exp, label_res=None):
    n = exp["n"]
    assert res["n"] == n and res["P"] == exp["P"]
    assert sha(res["M"]) == exp["M_sha256"]
    assert sha(res["sel"]) == exp["sel_sha256"]
    assert sha(res["allow"]) == exp["allow_sha256"]
    assert csr_sha(res["select_off"], res["select_list"]) == exp["select_policies_sha256"]
    assert csr_sha(res["allow_off"], res["allow_list"]) == exp["allow_policies_sha256"]
    assert res["all_reachable"] == exp["all_reachable"]
    assert res["all_isolated"] == exp["all_isolated"]
    if "result" in exp["user_crosscheck"]:
        assert res["user_crosscheck"] == exp["user_crosscheck"]["result"]
    assert res["system_isolation"] == exp["system_isolation"]["result"]
    assert res["shadow_count"] == exp["policy_shadow"]["count"]
    assert sha(res["shadow"].astype(np.int32)) == exp["policy_shadow"]["sha256"]
    assert res["conflict_raises"] == ("raises" in exp["policy_conflict"])
    if "M" in exp:
        assert words_to_rows01(res["M"], n) == exp["M"]


def test_paper_example_c_oracle():
    exp = expected("paper_example")
    res = orc.run_c(paper_json(), label="app")
    check_record(res, exp)
    assert exp["M"] == ["11010", "10010", "10010", "01000", "00100"]


@pytest.mark.parametrize("name", cluster_names())
def test_cluster_c_oracle(name):
    obj = cluster(name)
    exp = expected(name)
    res = orc.run_c(obj, label=obj.get("label", "app"))
    check_record(res, exp)


@pytest.mark.parametrize("name", [n for n in cluster_names()
                                  if n.startswith("q_") and n != "q_wide_select"] +
                         ["s_sparse_50"])   # (pure Python: the small full-matrix records)
def test_cluster_py_oracle(name):
    from kano.synth import objects_from_json
    from kano import model
    obj = cluster(name)
    exp = expected(name)
    cs, ps = objects_from_json(obj, model)
    res = orc.ref_py(cs, ps, label=obj.get("label", "app"))
    assert res["M"] == exp["M"]
    assert res["sel"] == exp["sel"] and res["allow"] == exp["allow"]
    assert res["select_policies"] == exp["select_policies"]
    assert res["allow_policies"] == exp["allow_policies"]
    assert res["all_reachable"] == exp["all_reachable"]
    assert res["all_isolated"] == exp["all_isolated"]
    assert res["user_crosscheck"] == exp["user_crosscheck"]["result"]
    assert res["system_isolation"] == exp["system_isolation"]["result"]
    assert [list(p) for p in res["policy_shadow"]] == exp["policy_shadow"]["all"]
    assert res["conflict_raises"] == ("raises" in exp["policy_conflict"])


def test_rebuilt_paper_lists_accumulate():
    """Quirk Q5: the second build appends again; shadow doubles."""
    exp = expected("paper_example_rebuilt")
    assert exp["select_policies"] == [[0, 3, 0, 3], [3, 3], [2, 3, 2, 3], [0, 0], [1, 1]]
    first = expected("paper_example")
    off, lst = lists_to_csr(exp["select_policies"])
    res = orc.run_c(paper_json(), label="app")
    # shadow over the accumulated lists with the same allow sets
    import ctypes
    cnt = ctypes.c_int64()
    n = 5
    out = np.zeros(2 * 64, np.int32)
    orc.lib().oracle_shadow(n, n, orc._p(off), orc._p(lst), orc._p(res["allow"]), 0, n, 64,
                            orc._p(out), ctypes.byref(cnt))
    assert cnt.value == exp["policy_shadow"]["count"] == 2 * 2 * first["policy_shadow"]["count"]
    assert out[: 2 * cnt.value].reshape(-1, 2).tolist() == exp["policy_shadow"]["all"]


@pytest.mark.slow
def test_c2_c_oracle():
    """C2 (10k pods / 1k policies, seed 0) against kano_py's hashes."""
    import os
    from _golden import GOLDEN
    path = os.path.join(GOLDEN, "expected", "C2.json")
    if not os.path.exists(path):
        pytest.skip("C2 golden not generated")
    from kano.synth import make_config
    exp = expected("C2")
    cl = make_config("C2")
    assert cl.fingerprint() == exp["seed"]["fingerprint"]
    obj = cl.to_json_obj()
    res = orc.run_c(obj, label="tenant")
    check_record(res, exp)


# --- policy_shadow's count without the list (C4) ----------------------------
def _count_cases():
    out = [n for n in cluster_names()] + ["C2"]
    out += sorted(f[:-5] for f in os.listdir(os.path.join(GOLDEN, "expected"))
                  if f.startswith("gen_") and expected(f[:-5])["n"] <= 10000)
    return out


def _obj(name):
    if name.startswith("gen_"):
        from refgen import cluster_json
        e = expected(name)
        g = e["generator"]
        return cluster_json(g["seed"], g["podN"], g["policyN"], e["walk_order"])
    if name in ("C2", "C3", "C4"):
        from kano.synth import make_config
        return make_config(name).to_json_obj()
    return cluster(name)


@pytest.mark.parametrize("name", _count_cases())
def test_shadow_count_grouped_vs_kano_py(name):
    """The grouped count restatement equals len(policy_shadow(...)) as
    kano_py computed it (algorithm.py:58-80)."""
    assert orc.shadow_count_grouped(_obj(name)) == expected(name)["policy_shadow"]["count"]


def test_big_config_counts_agree():
    """C3: kano_py's count and the oracle's agree; C4's count is the
    oracle's (make_golden.py --big + oracle_counts.py)."""
    for name in ("C3", "C4"):
        if not os.path.exists(os.path.join(GOLDEN, "expected", name + ".json")):
            pytest.fail(f"{name} golden missing (tests/golden/make_golden.py --big {name})")
        sh = expected(name)["policy_shadow"]
        assert "oracle_count" in sh
        if "count" in sh:
            assert sh["count"] == sh["oracle_count"]


# --- the reference generator (kano_py/tests/generate.py) --------------------
GEN = sorted(f[:-5] for f in os.listdir(os.path.join(GOLDEN, "expected"))
             if f.startswith("gen_"))


@pytest.mark.parametrize("name", GEN)
def test_refgen_reproduces_reference_generator(name):
    """The seeded restatement writes the same pods and YAML text as the
    reference's ConfigFiles after random.seed (digest recorded by
    make_golden.py --gen, which compared them file by file)."""
    from refgen import RefGen
    e = expected(name)
    g = e["generator"]
    rg = RefGen(g["seed"], podN=g["podN"], policyN=g["policyN"])
    assert rg.digest() == g["digest"]
    assert sorted(e["walk_order"]) == sorted(f for f, _ in rg.files)


@pytest.mark.parametrize("name", [n for n in GEN if expected(n)["n"] <= 1000])
def test_refgen_parsed_by_drop_in_parser(name, tmp_path):
    """The drop-in ConfigParser reads the generated files as kano_py's
    ConfigParser did (same select / allow dicts and directions, walk order
    replayed), and the C oracle on them reproduces kano_py's record."""
    from refgen import RefGen, cluster_json
    from kano.parser import ConfigParser
    e = expected(name)
    g = e["generator"]
    RefGen(g["seed"], podN=g["podN"], policyN=g["policyN"]).write(str(tmp_path))
    cp = ConfigParser()
    for f in e["walk_order"]:
        cp.parse(str(tmp_path / f))
    obj = cluster_json(g["seed"], g["podN"], g["policyN"], e["walk_order"])
    got = [(p.selector.labels, p.allow.labels, "ingress" if p.is_ingress() else "egress")
           for p in cp.policies]
    assert got == [(q["select"], q["allow"], q["direction"]) for q in obj["policies"]]
    res = orc.run_c(obj, label="User")
    check_record(res, e)
