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
    once (double kano_destroy)."""
    import gc
    from kano import _native as nat
    from kano._intern import tables_from_cluster
    from kano.multi import MultiBuild
    from kano.synth import make_config
    lib = nat.load()
    calls = {"ctx": 0, "group": 0}
    real_ctx, real_group = lib.kano_destroy, lib.kano_group_destroy

    def ctx_destroy(c):
        calls["ctx"] += 1
        return real_ctx(c)

    def group_destroy(g):
        calls["group"] += 1
        return real_group(g)
    monkeypatch.setattr(lib, "kano_destroy", ctx_destroy)
    monkeypatch.setattr(lib, "kano_group_destroy", group_destroy)
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
