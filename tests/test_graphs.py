"""kano_verify's operations recorded per segment and replayed as hipGraphs
(csrc/kano_graph.hpp; a knob, off by default: measured slower): a repeated step on one context is captured on its
second call and replayed from the third; the results must stay kano_py's
on every call, also when the inputs change between calls (new sequence ->
direct issue, then a new capture) and on row shards across the exchange."""
import numpy as np
import pytest

from _golden import cluster, expected, index_list_matches, sha

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from kano import _native
    if not _native.gpu_available():
        pytest.fail("GPU test run without a usable HIP device / libkano_hip.so")


def _tables(name):
    from kano._intern import intern, group_ids, tables_from_cluster
    from kano.synth import make_config, objects_from_json, KEY_NAMES
    from kano import model
    if name == "C2":
        cl = make_config("C2")
        gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1]
        return tables_from_cluster(cl), gid.astype(np.int32)
    obj = cluster(name)
    cs, ps = objects_from_json(obj, model)
    return intern(cs, ps), group_ids(cs, obj.get("label", "app"))


def _check(r, exp, pairs=True):
    assert index_list_matches(r["all_reachable"], exp["all_reachable"])
    assert index_list_matches(r["all_isolated"], exp["all_isolated"])
    assert index_list_matches(r["user_crosscheck"], exp["user_crosscheck"]["result"])
    assert index_list_matches(r["system_isolation"], exp["system_isolation"]["result"])
    assert r["shadow_count"] == exp["policy_shadow"]["count"]
    if pairs:
        assert sha(np.ascontiguousarray(r["pairs"], dtype=np.int32)) == \
            exp["policy_shadow"]["sha256"]


@pytest.mark.parametrize("name", ["C2", "s_sparse_2000", "s_broad_1000", "q_wide_select"])
def test_repeated_verify_replays_graphs(name, monkeypatch):
    from kano._engine import DeviceBuild, PinnedBuffer
    monkeypatch.setenv("KANO_TUNE", "graphs=1")
    t, gid = _tables(name)
    exp = expected(name)
    eng = DeviceBuild(t, build=False)
    eng.set_groups(gid)
    n = t.n
    pin = PinnedBuffer(8 * (1 << 20))
    idx = PinnedBuffer(4 * 4 * n)
    for step in range(6):
        r = eng.verify("stored", sys_row=0, shadow=True,
                       pairs=pin.view(np.int32, 2 << 20), idx=idx.view(np.int32, 4 * n))
        _check(r, exp)
        assert sha(eng.rows(0, n)) == exp["M_sha256"], f"step {step}"
        if step % 2:
            r = eng.verify("stored", sys_row=0, shadow=True, shadow_count_only=True)
            _check(r, exp, pairs=False)
    info = eng.info()
    assert info["GRAPH_HITS"] > 0 and info["GRAPH_CAPTURES"] > 0, info
    eng.close()
    pin.close()
    idx.close()


def test_inputs_change_between_calls(monkeypatch):
    """One context, the tables of three clusters in turn (each twice):
    every call gives its own cluster's results (a changed sequence never
    replays a stale graph)."""
    from kano._engine import DeviceBuild
    monkeypatch.setenv("KANO_TUNE", "graphs=1")
    eng = DeviceBuild(None)
    for name in ["s_sparse_2000", "C2", "s_sparse_2000", "q_wide_select", "C2",
                 "q_wide_select"]:
        t, gid = _tables(name)
        eng.upload(t)
        eng.set_groups(gid)
        for _ in range(3):
            r = eng.verify("stored", sys_row=0, shadow=True)
            _check(r, expected(name))
        assert sha(eng.rows(0, t.n)) == expected(name)["M_sha256"]
    eng.close()


def test_graphs_off_same_results(monkeypatch):
    from kano._engine import DeviceBuild
    monkeypatch.setenv("KANO_TUNE", "graphs=0")
    t, gid = _tables("C2")
    eng = DeviceBuild(t, build=False)
    eng.set_groups(gid)
    for _ in range(3):
        _check(eng.verify("stored", sys_row=0, shadow=True), expected("C2"))
    info = eng.info()
    assert info["GRAPH_HITS"] == 0 and info["GRAPH_CAPTURES"] == 0
    eng.close()
