"""One process over G devices (kano/multi.py, kano_group in the C ABI):
the UNCHANGED drop-in calls -- ReachabilityMatrix.build_matrix and every
kano.algorithm check -- on a matrix whose rows are split over G member
contexts, against kano_py's golden records.  KANO_NGPU = G selects the
group; KANO_DEVICES=0,0[,0] puts every member on cuda:0, so the exchange is
the device-copy form (the RCCL all-gather runs when the devices are
distinct, on an 8-GPU node)."""
import numpy as np
import pytest

from _golden import cluster, expected, sha

SHARD_CASES = ["paper_example", "s_sparse_2000", "s_broad_1000", "q_wide_select", "q_shadow",
               "q_dirs", "s_sparse_500", "q_types"]


def test_shard_bounds_are_word_aligned():
    from kano.multi import shard_bounds
    for n in (0, 1, 63, 64, 65, 1000, 100_000):
        for G in (1, 2, 3, 8):
            b = shard_bounds(n, G)
            assert b[0][0] == 0 and b[-1][1] == n
            for (a0, a1), (c0, _) in zip(b, b[1:]):
                assert a1 == c0 and a0 <= a1
            assert all(a % 64 == 0 for a, _ in b)


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("name", SHARD_CASES)
def test_drop_in_api_over_g_members(name, G, monkeypatch):
    from test_gpu_parity import api_objects, api_record, compare
    from kano.model import ReachabilityMatrix
    from kano.multi import MultiBuild
    monkeypatch.setenv("KANO_NGPU", str(G))
    monkeypatch.setenv("KANO_DEVICES", ",".join(["0"] * G))
    if name == "paper_example":
        from sample import paper_example
        cs, ps = paper_example()
        label = "app"
    else:
        obj = cluster(name)
        cs, ps = api_objects(obj)
        label = obj.get("label", "app")
    m = ReachabilityMatrix.build_matrix(cs, ps)
    assert isinstance(m.engine, MultiBuild) and m.engine.G == G
    assert m.engine.mode == "device copies"
    res = api_record(m, cs, ps, label)
    compare(res, expected(name))
    # system_isolation for a row of every member; getcol over all members
    from kano import algorithm as alg
    n = m.container_size
    M = res["M"]
    for i in sorted({0, n // 2, n - 1}):
        bits = np.unpackbits(M[i].view(np.uint8), bitorder="little")[:n]
        assert alg.system_isolation(m, i) == np.flatnonzero(bits == 0).tolist()
    for j in sorted({0, n - 1}):
        col = (M[:, j >> 6] >> np.uint64(j & 63)) & np.uint64(1)
        assert m.getcol(j).tolist() == col.astype(bool).tolist()
    m.engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3])
def test_group_verify_c2(G):
    """kano_group_verify (build + every check, one call over G members)
    against kano_py's C2 record, pairs and count-only."""
    from kano._intern import tables_from_cluster
    from kano.multi import MultiBuild
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
    eng = MultiBuild(tables_from_cluster(cl), G, devices=[0] * G, build=False)
    for _ in range(2):
        r = eng.verify(gid, sys_row=0, shadow=True)
        assert r["all_reachable"].tolist() == exp["all_reachable"]
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
        assert r["shadow_count"] == exp["policy_shadow"]["count"]
        assert sha(np.ascontiguousarray(r["pairs"])) == exp["policy_shadow"]["sha256"]
        assert sha(eng.rows(0, cl.n)) == exp["M_sha256"]
    c = eng.verify(gid, sys_row=cl.n - 1, shadow=True, shadow_count_only=True)
    assert c["shadow_count"] == exp["policy_shadow"]["count"] and c["pairs"] is None
    eng.close()


@pytest.mark.gpu
def test_group_verify_stored_groups_c2():
    """kano_group_set_groups + verify("stored") (the bench's form) against
    kano_py's C2 record."""
    from kano._intern import tables_from_cluster
    from kano.multi import MultiBuild
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
    eng = MultiBuild(tables_from_cluster(cl), 2, devices=[0, 0], build=False)
    eng.set_groups(gid)
    for _ in range(3):
        r = eng.verify("stored", sys_row=0, shadow=True)
        assert r["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
        assert sha(np.ascontiguousarray(r["pairs"])) == exp["policy_shadow"]["sha256"]
    eng.build()       # kano_group_build: every member at once
    assert sha(eng.rows(0, cl.n)) == exp["M_sha256"]
    eng.close()


@pytest.mark.gpu
def test_multibuild_failed_init_destroys_group_once(monkeypatch):
    """A failing upload inside MultiBuild.__init__: the adopted member
    wrappers never destroy their contexts, the group is destroyed exactly
    once (double kano_destroy).  Only this test's groups and
    members are counted (a collection may free earlier tests' engines)."""
    import gc
    from kano import _native as nat
    from kano._intern import tables_from_cluster
    from kano.multi import MultiBuild
    from kano.synth import make_config
    lib = nat.load()
    gc.collect()          # (earlier tests' engines in reference cycles: not ours)
    calls = {"ctx": 0, "group": 0}
    real_ctx, real_group = lib.kano_destroy, lib.kano_group_destroy
    real_member = lib.kano_group_member
    members = set()

    def member(g, r, out):
        rc = real_member(g, r, out)
        members.add(out._obj.value)
        return rc

    def ctx_destroy(c):
        if (c.value if hasattr(c, "value") else c) in members:
            calls["ctx"] += 1
        return real_ctx(c)

    real_create = lib.kano_group_create_ex
    groups = set()

    def group_create(ngpu, devs, flags, out):
        rc = real_create(ngpu, devs, flags, out)
        groups.add(out._obj.value)
        return rc

    def group_destroy(g):
        if (g.value if hasattr(g, "value") else g) in groups:
            calls["group"] += 1
        return real_group(g)
    monkeypatch.setattr(lib, "kano_destroy", ctx_destroy)
    monkeypatch.setattr(lib, "kano_group_destroy", group_destroy)
    monkeypatch.setattr(lib, "kano_group_member", member)
    monkeypatch.setattr(lib, "kano_group_create_ex", group_create)
    t = tables_from_cluster(make_config("C2"))
    import dataclasses
    bad = dataclasses.replace(t, sel_col=np.full_like(t.sel_col, t.ncols + 5))
    with pytest.raises(nat.KanoNativeError, match="term column out of range"):
        MultiBuild(bad, 2, devices=[0, 0])
    gc.collect()
    assert calls == {"ctx": 0, "group": 1}
    # the device is fine afterwards: a good group on the same tables
    eng = MultiBuild(t, 2, devices=[0, 0])
    assert eng.info()["U"] > 0
    eng.close()
    assert calls == {"ctx": 0, "group": 2}


@pytest.mark.gpu
def test_bench_group_line_two_members_one_device():
    """bench.py --gpus 2 without torch.distributed.run: one process, a
    kano_group of two members (KANO_DEVICES=0,0: device copies), one
    verified JSON line on C3."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, KANO_DEVICES="0,0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--steps", "20", "--warmup", "3"], capture_output=True, text=True,
                       timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["verified"] is True
    assert line["config"]["exchange"] == "device copies"
    assert line["config"]["devices"] == [0, 0]
    assert line["value"] > 0 and line["result_sizes"]["policy_shadow"] > 0


@pytest.mark.gpu
def test_group_rccl_transport_one_member():
    """The group's RCCL transport, run on one GPU: exchange="rccl" forces
    ncclCommInitAll over the member's device and the grouped ncclAllGather
    (issued from one thread, as for G distinct devices) for one member.
    kano_group_verify (pairs and count-only), kano_group_checks and
    kano_group_path then go through RCCL; results against kano_py's C2
    record (the column checks: kano_py/kano/algorithm.py:4-42)."""
    from kano import algorithm as alg
    from kano._intern import tables_from_cluster
    from kano.model import ReachabilityMatrix
    from kano.multi import MultiBuild
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
    eng = MultiBuild(tables_from_cluster(cl), 1, devices=[0], build=False, exchange="rccl")
    info = np.zeros(2, dtype=np.int32)
    eng.lib.kano_group_info(eng.g, info.ctypes.data)
    assert int(info[1]) == 1 and eng.mode == "rccl all-gather"
    eng.exchange_timing(enable=True, reset=True)
    eng.set_groups(gid)
    for g in (gid, "stored"):
        r = eng.verify(g, sys_row=0, shadow=True)
        assert r["all_reachable"].tolist() == exp["all_reachable"]
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
        assert sha(np.ascontiguousarray(r["pairs"])) == exp["policy_shadow"]["sha256"]
    c = eng.verify(gid, sys_row=0, shadow=True, shadow_count_only=True)
    assert c["shadow_count"] == exp["policy_shadow"]["count"]
    xt = eng.exchange_timing()
    assert xt["calls"] == 3 and xt["total_ms"] > 0
    assert sha(eng.rows(0, cl.n)) == exp["M_sha256"]
    chk = eng.checks(gid, sys_row=0)
    assert chk["all_isolated"].tolist() == exp["all_isolated"]
    assert chk["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
    # kano_group_path over the same transport, against the single-device path
    m = ReachabilityMatrix.__new__(ReachabilityMatrix)
    m.container_size, m._engine, m._lists = cl.n, eng, None
    two = alg.two_hop(m)
    assert isinstance(two.engine, MultiBuild)
    from kano._engine import DeviceBuild
    single = DeviceBuild(tables_from_cluster(cl))
    ref = DeviceBuild.empty(cl.n)
    ref.path_from(single, hops=2)
    assert np.array_equal(two.engine.rows(0, cl.n), ref.rows(0, cl.n))
    for e in (two.engine, ref, single, eng):
        e.close()


@pytest.mark.gpu
def test_group_rccl_failure_is_loud(monkeypatch):
    """An RCCL exchange that cannot run is an error with its reason, never a
    silent fall back to device copies: RCCL asked for over members sharing
    a device (ncclCommInitAll needs distinct devices)."""
    from kano import _native as nat
    from kano._intern import tables_from_cluster
    from kano.multi import MultiBuild
    from kano.synth import make_config
    t = tables_from_cluster(make_config("C2"))
    with pytest.raises(nat.KanoNativeError, match="distinct devices"):
        MultiBuild(t, 2, devices=[0, 0], exchange="rccl")
    monkeypatch.setenv("KANO_GROUP_RCCL", "1")
    with pytest.raises(nat.KanoNativeError, match="distinct devices"):
        MultiBuild(t, 2, devices=[0, 0])
    monkeypatch.delenv("KANO_GROUP_RCCL")
    eng = MultiBuild(t, 2, devices=[0, 0])      # copies: the devices are shared
    assert eng.mode == "device copies"
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["s_sparse_1000", "s_broad_300", "q_wide_select"])
def test_drop_in_incremental_over_g_members(name, monkeypatch):
    """ReachabilityMatrix.remove_policies / add_policies on a matrix split
    over two members (kano_group_remove_policies / _add_policies), against
    the oracle over the updated policy list (kano_py/kano/model.py:125-165)."""
    from test_incremental import _check_vs_oracle, _objs, _oracle, _policy
    from kano import model
    from kano.model import ReachabilityMatrix
    from kano.multi import MultiBuild
    monkeypatch.setenv("KANO_NGPU", "2")
    monkeypatch.setenv("KANO_DEVICES", "0,0")
    obj = cluster(name)
    label = obj.get("label", "app")
    cs, ps = _objs(obj)
    P = len(ps)
    gone = sorted({0, P // 3, P - 1})
    keep = [p for p in range(P) if p not in gone]
    m = ReachabilityMatrix.build_matrix(cs, ps)
    assert isinstance(m.engine, MultiBuild)
    m.remove_policies(gone)
    _check_vs_oracle(m, cs, ps, _oracle(obj, keep), label)
    back = [obj["policies"][gone[0]], obj["policies"][gone[-1]]]
    m.add_policies([_policy(model, q) for q in back])
    _check_vs_oracle(m, cs, ps, _oracle(obj, keep, back), label)
    m.engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("hops", [2, 0])
def test_drop_in_path_over_g_members(G, hops, monkeypatch):
    """kano.algorithm.two_hop / transitive_closure on a matrix split over G
    members (kano_group_path: one exchange of the one-hop table parts),
    against the oracle's path matrix (kubesv constraint.py:233-237 restated)."""
    from kano import algorithm as alg
    from kano.model import ReachabilityMatrix
    from kano.multi import MultiBuild
    from oracle import kano_oracle as orc
    monkeypatch.setenv("KANO_NGPU", str(G))
    monkeypatch.setenv("KANO_DEVICES", ",".join(["0"] * G))
    from test_gpu_parity import api_objects
    obj = cluster("s_sparse_2000")
    cs, ps = api_objects(obj)
    m = ReachabilityMatrix.build_matrix(cs, ps)
    assert isinstance(m.engine, MultiBuild)
    n = m.container_size
    ref, _ = orc.path_c(m.engine.rows(0, n), n, hops)
    out = alg.two_hop(m) if hops == 2 else alg.transitive_closure(m)
    assert isinstance(out.engine, MultiBuild) and out.engine.G == G
    assert np.array_equal(out.engine.rows(0, n), ref)
    # a whole-matrix check on the sharded path matrix (the group's exchange)
    col_or = np.bitwise_or.reduce(ref, axis=0)
    bits = np.unpackbits(col_or.view(np.uint8), bitorder="little")[:n]
    assert alg.all_isolated(out) == np.flatnonzero(bits == 0).tolist()
    out.engine.close()
    m.engine.close()
