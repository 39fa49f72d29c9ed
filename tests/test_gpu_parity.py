"""GPU parity: the HIP engine (through the C ABI and the drop-in API) against
kano_py's golden vectors and the C oracle.  Bit-exact everywhere."""
import os

import numpy as np
import pytest

from _golden import (cluster, cluster_names, csr_sha, expected, lists_to_csr, sha,
                     words_to_rows01)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from kano import _native
    if not _native.gpu_available():
        pytest.fail("GPU test run without a usable HIP device / libkano_hip.so")


def api_objects(obj):
    from kano import model
    from kano.synth import objects_from_json
    return objects_from_json(obj, model)


def api_record(m, cs, ps, label):
    """Run every query through the drop-in API; canonical layouts."""
    from kano import algorithm as alg
    n = m.container_size
    res = {"n": n, "P": len(ps)}
    res["M"] = m.engine.rows(0, n) if n else np.zeros((0, 1), np.uint64)
    res["sel"] = np.array([p.working_select_set.words() for p in ps]).reshape(len(ps), -1)
    res["allow"] = np.array([p.working_allow_set.words() for p in ps]).reshape(len(ps), -1)
    res["select_csr"] = lists_to_csr([c.select_policies for c in cs])
    res["allow_csr"] = lists_to_csr([c.allow_policies for c in cs])
    res["all_reachable"] = alg.all_reachable(m)
    res["all_isolated"] = alg.all_isolated(m)
    res["user_crosscheck"] = alg.user_crosscheck(m, cs, label)
    res["system_isolation"] = alg.system_isolation(m, 0) if n else []
    res["policy_shadow"] = alg.policy_shadow(m, ps, cs)
    try:
        res["policy_conflict"] = ("ok", alg.policy_conflict(m, ps, cs))
    except AttributeError as e:
        res["policy_conflict"] = ("raises", str(e))
    return res


def compare(res, exp):
    n = exp["n"]
    assert sha(res["M"]) == exp["M_sha256"]
    if "M" in exp:
        assert words_to_rows01(res["M"], n) == exp["M"]
    assert sha(res["sel"]) == exp["sel_sha256"]
    assert sha(res["allow"]) == exp["allow_sha256"]
    assert csr_sha(*res["select_csr"]) == exp["select_policies_sha256"]
    assert csr_sha(*res["allow_csr"]) == exp["allow_policies_sha256"]
    assert res["all_reachable"] == exp["all_reachable"]
    assert res["all_isolated"] == exp["all_isolated"]
    assert res["user_crosscheck"] == exp["user_crosscheck"]["result"]
    assert res["system_isolation"] == exp["system_isolation"]["result"]
    pairs = res["policy_shadow"]
    assert len(pairs) == exp["policy_shadow"]["count"]
    assert sha(np.array(pairs, np.int32).reshape(-1, 2)) == exp["policy_shadow"]["sha256"]
    if "raises" in exp["policy_conflict"]:
        assert res["policy_conflict"] == ("raises", exp["policy_conflict"]["message"])
    else:
        assert res["policy_conflict"] == ("ok", exp["policy_conflict"]["result"])


def test_paper_example_known_answers():
    """kano_py/tests/test_basic.py:28-37 with paper_example."""
    from sample import paper_example
    from kano.model import ReachabilityMatrix
    from kano.algorithm import (all_isolated, all_reachable, policy_conflict, policy_shadow,
                                system_isolation, user_crosscheck)
    cs, ps = paper_example()
    m = ReachabilityMatrix.build_matrix(cs, ps)
    assert m[0, 1] & m[2, 0] & m[4, 2]
    assert all_reachable(m) == []
    assert all_isolated(m) == [4]
    assert user_crosscheck(m, cs, "app") == [1, 2, 3]
    assert policy_shadow(m, ps, cs) == [(2, 3), (3, 2)]
    assert system_isolation(m, 0) == [2, 4]
    assert [r.to01() for r in m.matrix] == ["11010", "10010", "10010", "01000", "00100"]
    assert [p.working_select_set.to01() for p in ps] == ["10010", "00001", "00100", "11100"]
    assert [p.working_allow_set.to01() for p in ps] == ["01000", "00100", "10010", "10010"]
    assert [c.select_policies for c in cs] == [[0, 3], [3], [2, 3], [0], [1]]
    assert [c.allow_policies for c in cs] == [[2, 3], [0], [1], [2, 3], []]
    assert m.getcol(0).to01() == "11100" and m.getrow(3).to01() == "01000"
    with pytest.raises(AttributeError, match="'int' object has no attribute 'working_allow_set'"):
        policy_conflict(m, ps, cs)
    compare(api_record(m, cs, ps, "app"), expected("paper_example"))


def test_paper_example_rebuilt_accumulates():
    """Quirk Q5: a second build on the same objects appends again, and
    policy_shadow then runs on the accumulated lists."""
    from sample import paper_example
    from kano.model import ReachabilityMatrix
    cs, ps = paper_example()
    ReachabilityMatrix.build_matrix(cs, ps)
    m2 = ReachabilityMatrix.build_matrix(cs, ps)
    compare(api_record(m2, cs, ps, "app"), expected("paper_example_rebuilt"))


@pytest.mark.parametrize("name", cluster_names())
def test_golden_cluster_api(name):
    from kano.model import ReachabilityMatrix
    obj = cluster(name)
    cs, ps = api_objects(obj)
    m = ReachabilityMatrix.build_matrix(cs, ps)
    compare(api_record(m, cs, ps, obj.get("label", "app")), expected(name))


@pytest.mark.parametrize("name", ["s_broad_300", "s_broad_1000", "s_sparse_1000",
                                  "s_sparse_2000", "q_dirs", "q_shadow"])
@pytest.mark.parametrize("path", ["bitwise", "mfma", "auto", "mfma-gemm22", "mfma-gemm42",
                                  "mfma-gemm44", "mfma-dx", "mfma-dx22", "bitwise-dx"])
def test_build_paths_agree(name, path, monkeypatch):
    """The bitwise (LDS scatter / OR) and fp4-MFMA contraction paths -- the
    split-K kernel and the tiled GEMM in its three wave tiles, forced at
    these sizes (hgemmmin=1) -- give kano_py's matrix and column checks."""
    from kano._engine import DeviceBuild
    from kano._intern import intern
    if path == "mfma-dx":    # the dense path's bit matrices; A is SA as it stands
        monkeypatch.setenv("KANO_TUNE", "dx=2,hgemm=44,hgemmmin=1")
        path = "mfma"
    if path == "mfma-dx22":  # the same on the 2 x 2 tile (A is SA when its pitch fits)
        monkeypatch.setenv("KANO_TUNE", "dx=2,hgemm=22,hgemmmin=1")
        path = "mfma"
    if path == "bitwise-dx":
        monkeypatch.setenv("KANO_TUNE", "dx=2")
        path = "bitwise"
    if path.startswith("mfma-gemm"):
        tile = path[len("mfma-gemm"):len("mfma-gemm") + 2]
        monkeypatch.setenv("KANO_TUNE", f"hgemm={tile},hgemmmin=1")
        path = "mfma"
    obj = cluster(name)
    cs, ps = api_objects(obj)
    exp = expected(name)
    eng = DeviceBuild(intern(cs, ps), path=path)
    n = len(cs)
    assert sha(eng.rows(0, n)) == exp["M_sha256"]
    ca, co = eng.col_checks()
    from kano._bits import set_bit_indices, words_to_bool
    assert set_bit_indices(ca, n).tolist() == exp["all_reachable"]
    assert np.flatnonzero(~words_to_bool(co, n)).tolist() == exp["all_isolated"]
    if path == "mfma":
        assert eng.info()["HEAVY"] > 0 or exp["P"] == 0
        assert eng.info()["HEAVY_PATH"] == 2 or exp["P"] == 0
    eng.close()


def test_c2_engine_vs_kano_py():
    """C2 (BASELINE configs[1]: 10k pods / 1k policies, seed 0) bit-exact
    against kano_py's hashes, through the direct-table path of the bench."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano._bits import set_bit_indices, words_to_bool
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    assert cl.fingerprint() == exp["seed"]["fingerprint"]
    eng = DeviceBuild(tables_from_cluster(cl))
    n = cl.n
    assert sha(eng.rows(0, n)) == exp["M_sha256"]
    ca, co = eng.col_checks()
    assert set_bit_indices(ca, n).tolist() == exp["all_reachable"]
    assert np.flatnonzero(~words_to_bool(co, n)).tolist() == exp["all_isolated"]
    gid = cl.vals[KEY_NAMES.index("tenant")]
    _, gid = np.unique(gid, return_inverse=True)
    assert set_bit_indices(eng.crosscheck(gid), n).tolist() == exp["user_crosscheck"]["result"]
    pairs = eng.shadow()
    assert pairs.shape[0] == exp["policy_shadow"]["count"]
    assert sha(pairs) == exp["policy_shadow"]["sha256"]
    row0 = eng.rows(0, 1)[0]
    assert np.flatnonzero(~words_to_bool(row0, n)).tolist() == exp["system_isolation"]["result"]
    eng.close()


@pytest.mark.parametrize("cap", [0, 1 << 22])
def test_verify_fused_c2(cap):
    """kano_verify (build + every check in one call, the bench's step) gives
    kano_py's result lists on C2; cap=0 exercises the late pair fetch."""
    from kano._engine import DeviceBuild, PinnedBuffer
    from kano._intern import tables_from_cluster
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    n = cl.n
    _, gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    pin = PinnedBuffer(max(cap, 1) * 8)
    eng.set_groups(gid)
    for g, ng in ((gid, 0), (gid, int(gid.max()) + 1), ("stored", 0)):
        # host-scanned / declared group count / groups stored on the device
        r = eng.verify(g, sys_row=0, shadow=True, ngroups=ng,
                       pairs=pin.view(np.int32, 2 * cap) if cap else None)
        assert sha(eng.rows(0, n)) == exp["M_sha256"]
        assert r["all_reachable"].tolist() == exp["all_reachable"]
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
        assert r["shadow_count"] == exp["policy_shadow"]["count"]
        assert sha(np.ascontiguousarray(r["pairs"])) == exp["policy_shadow"]["sha256"]
    eng.close()
    pin.close()


@pytest.mark.parametrize("tune", ["", "xcdmin=0", "xcdmin=0,xcdside=0", "xcdmin=0,xcdside=1"])
def test_verify_pipelined(tune, monkeypatch):
    """kano_set_pipeline: every asynchronously completing verify queues the
    next call's prologue behind a gate the next verify opens.  Every call's
    results equal kano_py's (C2's record) whatever comes between two calls:
    nothing, a matrix read, a re-upload, another cluster's tables, a plain
    build, a pause past the gate's timeout (the prologue then ran by itself on
    the same inputs), count-only mode, the emulated shard path, the pipeline
    switched off while a prologue is queued, and a close while one is queued.
    xcdmin=0: the XCD split at C2's size (the engine stream on XCDs 3-7, the
    write on 0-2, switched between calls as the last write qualifies);
    xcdside=0 / 1 keep the side stream unmasked / move it with the engine
    stream whatever the last build's heavy classes."""
    if tune:
        monkeypatch.setenv("KANO_TUNE", tune)
    import time
    import torch
    from kano._engine import DeviceBuild, PinnedBuffer
    from kano._intern import tables_from_cluster, intern, group_ids
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    n = cl.n
    _, gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)
    tables = tables_from_cluster(cl)
    eng = DeviceBuild(tables, build=False)
    eng.set_pipeline(True)
    pin = PinnedBuffer((1 << 22) * 8)
    pairs = pin.view(np.int32, 2 << 22)
    eng.set_groups(gid)

    def check(r, e=exp, count_only=False):
        assert r["all_isolated"].tolist() == e["all_isolated"]
        assert r["all_reachable"].tolist() == e["all_reachable"]
        assert r["user_crosscheck"].tolist() == e["user_crosscheck"]["result"]
        assert r["shadow_count"] == e["policy_shadow"]["count"]
        if not count_only:
            assert sha(np.ascontiguousarray(r["pairs"])) == e["policy_shadow"]["sha256"]

    for k in range(10):
        r = eng.verify("stored", sys_row=0, shadow=True, pairs=pairs)
        check(r)
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
        if k == 2:
            assert sha(eng.rows(0, n)) == exp["M_sha256"]    # (unprimes, then reads)
        if k == 4:
            eng.upload(tables)
            eng.set_groups(gid)
        if k == 5:
            time.sleep(0.35)     # past the gate's 200 ms: the prologue ran by itself
        if k == 6:
            eng.build()          # a plain build takes no primed prologue
            assert sha(eng.rows(0, n)) == exp["M_sha256"]
        if k == 7:
            r = eng.verify("stored", sys_row=0, shadow=True, shadow_count_only=True)
            check(r, count_only=True)
    assert sha(eng.rows(0, n)) == exp["M_sha256"]
    # another cluster's tables right behind a primed call, and back
    r = eng.verify("stored", sys_row=0, shadow=True, pairs=pairs)
    obj = cluster("s_sparse_2000")
    cs, ps = api_objects(obj)
    eng.upload(intern(cs, ps))
    e2 = expected("s_sparse_2000")
    for _ in range(3):
        rb = eng.verify(group_ids(cs, obj["label"]), sys_row=0, shadow=True, pairs=pairs)
        assert rb["all_isolated"].tolist() == e2["all_isolated"]
        assert rb["user_crosscheck"].tolist() == e2["user_crosscheck"]["result"]
        assert rb["shadow_count"] == e2["policy_shadow"]["count"]
    assert sha(eng.rows(0, len(cs))) == e2["M_sha256"]
    eng.upload(tables)
    eng.set_groups(gid)
    for _ in range(3):
        check(eng.verify("stored", sys_row=0, shadow=True, pairs=pairs))
    # settle: nothing of the engine left on the device, so a device-wide
    # synchronisation returns at once (no gate's timeout)
    eng.settle()
    t = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t < 0.1
    check(eng.verify("stored", sys_row=0, shadow=True, pairs=pairs))
    eng.set_pipeline(False)          # with a prologue queued
    check(eng.verify("stored", sys_row=0, shadow=True, pairs=pairs))
    eng.set_pipeline(True)
    check(eng.verify("stored", sys_row=0, shadow=True, pairs=pairs))
    t = time.perf_counter()
    eng.close()                      # with a prologue queued: opens its gate
    assert time.perf_counter() - t < 0.15
    # the emulated shard path (kano_verify_gather, comm NULL) pipelined: its
    # rows and pairs equal the unpipelined call's
    ref = DeviceBuild(tables, rows=(0, n // 4), build=False)
    ref.set_groups(gid)
    r0 = ref.verify_gather(0, 4, gid="stored", sys_row=0, shadow=True)
    r0 = {k: (np.array(v, copy=True) if v is not None else None) for k, v in r0.items()}
    d0 = ref.rows_digest(0, n // 4)
    ref.close()
    e = DeviceBuild(tables, rows=(0, n // 4), build=False)
    e.set_groups(gid)
    e.set_pipeline(True)
    for _ in range(4):
        r = e.verify_gather(0, 4, gid="stored", sys_row=0, shadow=True)
        for key in ("all_isolated", "user_crosscheck", "system_isolation", "pairs"):
            assert np.array_equal(r[key], r0[key]), key
    assert np.array_equal(e.rows_digest(0, n // 4), d0)
    e.close()
    pin.close()


@pytest.mark.parametrize("tune", ["async=1", "async=0"])
def test_verify_async_completion(tune, monkeypatch):
    """kano_verify returns once its host results are in host memory, its
    matrix write still queued (async=1, the default): back-to-back calls, a
    matrix read right after, an upload between calls, a two-hop product
    reading the source's matrix from another context and the k_rows timing
    all see the finished matrix."""
    monkeypatch.setenv("KANO_TUNE", tune)
    from kano._engine import DeviceBuild, PinnedBuffer
    from kano._intern import tables_from_cluster
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    n = cl.n
    _, gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)
    tables = tables_from_cluster(cl)
    eng = DeviceBuild(tables, build=False)
    pin = PinnedBuffer((1 << 22) * 8)
    pairs = pin.view(np.int32, 2 << 22)
    eng.set_groups(gid)
    eng.rows_timing(reset=True)
    for k in range(4):
        r = eng.verify("stored", sys_row=0, shadow=True, pairs=pairs)
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["shadow_count"] == exp["policy_shadow"]["count"]
        assert sha(np.ascontiguousarray(r["pairs"])) == exp["policy_shadow"]["sha256"]
        if k == 1:
            assert sha(eng.rows(0, n)) == exp["M_sha256"]
        if k == 2:
            eng.upload(tables)          # an upload between two calls
            eng.set_groups(gid)
    rt = eng.rows_timing()
    assert rt["launches"] == 4 and 0 < rt["min_ms"] <= rt["max_ms"]
    assert sha(eng.rows(0, n)) == exp["M_sha256"]
    r = eng.verify("stored", sys_row=0, shadow=True, pairs=pairs)
    # another context reads this one's matrix right after the call (one hop
    # of kano_path: the matrix itself)
    dst = DeviceBuild.empty(n)
    info = np.zeros(8, dtype=np.int64)
    assert eng.lib.kano_path(eng.ctx, dst.ctx, 1, 0, info.ctypes.data) == 0
    assert sha(dst.rows(0, n)) == exp["M_sha256"]
    dst.close()
    # other clusters on the same context right behind an asynchronously
    # completing call: their builds reallocate buffers the previous matrix
    # write may still read (2k pods, then C2's 10k again)
    from kano._intern import intern, group_ids
    r = eng.verify("stored", sys_row=0, shadow=True, pairs=pairs)
    obj = cluster("s_sparse_2000")
    cs, ps = api_objects(obj)
    eng.upload(intern(cs, ps))
    rb = eng.verify(group_ids(cs, obj["label"]), sys_row=0, shadow=True, pairs=pairs)
    e2 = expected("s_sparse_2000")
    assert rb["all_isolated"].tolist() == e2["all_isolated"]
    assert rb["user_crosscheck"].tolist() == e2["user_crosscheck"]["result"]
    assert rb["shadow_count"] == e2["policy_shadow"]["count"]
    eng.upload(tables)
    eng.set_groups(gid)
    r = eng.verify("stored", sys_row=0, shadow=True, pairs=pairs)
    assert r["all_isolated"].tolist() == exp["all_isolated"]
    assert sha(eng.rows(0, n)) == exp["M_sha256"]
    eng.close()
    pin.close()


def test_verify_pairs_then_fetch():
    """policy_shadow's pairs returned by kano_verify, a kano_shadow_fetch after
    the call, and a buffer too small for them (the pairs then come from the
    device through kano_shadow_fetch) all match kano_py's C2 record."""
    from kano._engine import DeviceBuild, PinnedBuffer
    from kano._intern import tables_from_cluster
    from kano.synth import make_config, KEY_NAMES
    exp = expected("C2")
    cl = make_config("C2")
    _, gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    eng.set_groups(gid)
    want = exp["policy_shadow"]
    k = want["count"]
    assert k > 16
    big = PinnedBuffer((k + 64) * 8)
    small = PinnedBuffer(16 * 8)
    for _ in range(2):
        r = eng.verify("stored", sys_row=0, shadow=True, pairs=big.view(np.int32, 2 * (k + 64)))
        assert r["shadow_count"] == k
        assert sha(np.ascontiguousarray(r["pairs"])) == want["sha256"]
        assert sha(np.ascontiguousarray(eng.shadow_fetch(k))) == want["sha256"]
        r = eng.verify("stored", sys_row=0, shadow=True, pairs=small.view(np.int32, 32))
        assert r["shadow_count"] == k
        assert sha(np.ascontiguousarray(r["pairs"])) == want["sha256"]
    eng.close()
    big.close()
    small.close()


def test_verify_status_regions_after_a_smaller_call():
    """k_verify_cols_f's look-back status regions (two, alternating) on one
    context: a large call, a small call, then a DIFFERENT cluster at the
    large size.  The third call reads the region the first call used; every
    word of it must have been cleared (only the small call's
    prefix was, and stale look-back prefixes of the first cluster survived)."""
    from kano._engine import DeviceBuild
    from kano._intern import group_ids, intern, tables_from_cluster
    from kano.synth import make_cluster, make_config, KEY_NAMES
    from oracle import kano_oracle as orc
    cl = make_config("C2")
    _, gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    r = eng.verify(gid, sys_row=0, shadow=False)
    assert r["all_isolated"].tolist() == expected("C2")["all_isolated"]
    small = cluster("s_sparse_500")
    cs, ps = api_objects(small)
    eng.upload(intern(cs, ps))
    r = eng.verify(group_ids(cs, small["label"]), sys_row=0, shadow=False)
    assert r["user_crosscheck"].tolist() == expected("s_sparse_500")["user_crosscheck"]["result"]
    other = make_cluster(10_000, 1_000, "sparse", seed=123).to_json_obj()
    ref = orc.run_c(other, label="tenant")
    cs, ps = api_objects(other)
    eng.upload(intern(cs, ps))
    for _ in range(2):
        r = eng.verify(group_ids(cs, "tenant"), sys_row=0, shadow=True)
        assert r["all_reachable"].tolist() == ref["all_reachable"]
        assert r["all_isolated"].tolist() == ref["all_isolated"]
        assert r["user_crosscheck"].tolist() == ref["user_crosscheck"]
        assert r["system_isolation"].tolist() == ref["system_isolation"]
        assert np.array_equal(np.ascontiguousarray(r["pairs"]).reshape(-1, 2),
                              ref["shadow"].reshape(-1, 2))
    eng.close()


def test_build_matrix_closes_engine_when_build_raises(monkeypatch):
    """ReachabilityMatrix.build_matrix whose upload or build raises destroys
    the context it made (no device memory left until GC)."""
    import gc
    from kano import _native as nat
    from kano._engine import DeviceBuild
    from kano.model import ReachabilityMatrix
    lib = nat.load()
    made, destroyed = [], []
    real_create, real_destroy = lib.kano_create_lean, lib.kano_destroy

    def create(dev, out):
        made.append(dev)
        return real_create(dev, out)

    def destroy(c):
        destroyed.append(c)
        return real_destroy(c)
    monkeypatch.setattr(lib, "kano_create_lean", create)
    monkeypatch.setattr(lib, "kano_destroy", destroy)
    cs, ps = api_objects(cluster("s_sparse_200"))
    for what in ("upload", "build"):
        def boom(self, *a, **k):
            raise nat.KanoNativeError(f"injected {what} failure")
        monkeypatch.setattr(DeviceBuild, what, boom)
        gc.disable()
        try:
            ReachabilityMatrix.build_matrix(cs, ps)
            raise AssertionError("build_matrix did not raise")
        except nat.KanoNativeError as e:
            assert "injected" in str(e)
            # (checked while the traceback, and every frame's engine, lives)
            assert len(destroyed) == len(made), (what, made, destroyed)
        finally:
            gc.enable()
        monkeypatch.undo()
        monkeypatch.setattr(lib, "kano_create_lean", create)
        monkeypatch.setattr(lib, "kano_destroy", destroy)
    assert len(made) == 2


def test_lists_follow_the_build_order_after_reordering():
    """The containers' lists belong to the build's order even when the caller
    reorders, pops or inserts into its list after build_matrix (ADVICE r4:
    the lists were mapped through the live list on first use); policy_shadow
    then iterates the containers in their new order (algorithm.py:58-80)."""
    from kano import algorithm as alg
    from kano.model import ReachabilityMatrix
    obj = cluster("s_sparse_200")
    exp = expected("s_sparse_200")
    cs, ps = api_objects(obj)
    build_order = list(cs)
    m = ReachabilityMatrix.build_matrix(cs, ps)
    cs.reverse()
    cs.pop(0)
    cs.insert(3, cs[10])
    sel = exp["select_policies"]
    pos = {id(c): i for i, c in enumerate(build_order)}
    for c in cs:
        assert c.select_policies == sel[pos[id(c)]]
        assert c.allow_policies == exp["allow_policies"][pos[id(c)]]
    # policy_shadow over the reordered list: kano_py's loop on these lists
    allow = [{i for i, ch in enumerate(a) if ch == "1"} for a in exp["allow"]]
    want = [(j, k) for c in cs for j in c.select_policies for k in c.select_policies
            if j != k and allow[k] <= allow[j]]
    assert alg.policy_shadow(m, ps, cs) == want
    m.engine.close()


def test_verify_declared_groups_checked():
    """A group id outside the declared [0, ngroups) is an error, not a fault
    (the check in k_cls_group_range_m)."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    from kano._native import KanoNativeError
    obj = cluster("s_sparse_1000")
    cs, ps = api_objects(obj)
    gid = group_ids(cs, obj["label"])
    eng = DeviceBuild(intern(cs, ps), build=False)
    with pytest.raises(KanoNativeError, match="ngroups"):
        eng.verify(gid, ngroups=max(1, int(gid.max())), shadow=False)
    r = eng.verify(gid, ngroups=int(gid.max()) + 1, shadow=False)
    assert r["user_crosscheck"].tolist() == expected("s_sparse_1000")["user_crosscheck"]["result"]
    eng.close()


@pytest.mark.parametrize("name", ["paper_example", "q_dirs", "s_broad_300"])
def test_verify_fused_golden(name):
    """kano_verify without a group label and without policy_shadow."""
    from kano._engine import DeviceBuild
    from kano._intern import intern
    if name == "paper_example":
        from sample import paper_example
        cs, ps = paper_example()
    else:
        cs, ps = api_objects(cluster(name))
    exp = expected(name)
    eng = DeviceBuild(intern(cs, ps), build=False)
    r = eng.verify(None, sys_row=0, shadow=False)
    assert r["all_reachable"].tolist() == exp["all_reachable"]
    assert r["all_isolated"].tolist() == exp["all_isolated"]
    assert r["user_crosscheck"] is None and "pairs" not in r
    if len(cs):
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
    eng.close()


def test_verify_fused_shards():
    """kano_verify on row shards: per-shard pairs concatenate to the full
    list, per-shard crosscheck lists union to the full one, the system row
    comes only from its owner."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    from oracle import kano_oracle as orc
    obj = cluster("s_sparse_2000")
    cs, ps = api_objects(obj)
    t = intern(cs, ps)
    n = len(cs)
    ref = orc.run_c(obj, label=obj["label"])
    gid = group_ids(cs, obj["label"])
    pairs, cross = [], set()
    for r0, r1 in [(0, 700), (700, n)]:
        e = DeviceBuild(t, rows=(r0, r1), build=False)
        r = e.verify(gid, sys_row=5, shadow=True)
        pairs.append(r["pairs"])
        cross |= set(r["user_crosscheck"].tolist())
        if r0 <= 5 < r1:
            from kano._bits import words_to_bool
            row = e.rows(5, 1)[0]
            assert r["system_isolation"].tolist() == np.flatnonzero(
                ~words_to_bool(row, n)).tolist()
        else:
            assert r["system_isolation"] is None
        e.close()
    assert np.array_equal(np.concatenate(pairs), ref["shadow"])
    assert sorted(cross) == ref["user_crosscheck"]


@pytest.mark.parametrize("name,spans", [
    ("s_sparse_2000", [(0, 700), (700, 2000)]),
    ("s_sparse_2000", [(0, 0), (0, 1), (1, 1300), (1300, 2000)]),   # empty shards
    ("C2", [(k * 10000 // 8, (k + 1) * 10000 // 8) for k in range(8)]),
    ("s_broad_1000", [(0, 333), (333, 667), (667, 1000)]),
])
def test_verify_shard_combine(name, spans):
    """The multi-GPU step on one device: every shard runs kano_verify_shard
    into its slot of one gathered word buffer (what the RCCL all-gather
    builds), then kano_verify_combine gives the full column lists on every
    shard, the system row on its owner, and pairs that concatenate in shard
    order to the reference's list."""
    import torch
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids, tables_from_cluster
    from kano.synth import make_config, KEY_NAMES
    if name == "C2":
        cl = make_config("C2")
        t = tables_from_cluster(cl)
        gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
    else:
        obj = cluster(name)
        cs, ps = api_objects(obj)
        t = intern(cs, ps)
        gid = group_ids(cs, obj["label"])
    exp = expected(name)
    n = t.n
    W = (n + 63) // 64
    N = len(spans)
    assert spans[0][0] == 0 and spans[-1][1] == n
    gathered = torch.zeros(N * 3 * W, dtype=torch.int64, device="cuda")
    engs = [DeviceBuild(t, rows=s, build=False) for s in spans]
    for k, e in enumerate(engs):
        e.verify_shard(gathered.data_ptr() + 8 * 3 * W * k, gid=gid, sys_row=0, shadow=True)
    torch.cuda.synchronize()
    pairs = []
    for k, (e, (r0, r1)) in enumerate(zip(engs, spans)):
        r = e.verify_combine(gathered.data_ptr(), N)
        assert r["all_reachable"].tolist() == exp["all_reachable"]
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
        if r0 <= 0 < r1:
            assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
        else:
            assert r["system_isolation"] is None
        pairs.append(np.ascontiguousarray(r["pairs"]).reshape(-1, 2))
        e.close()
    allp = np.ascontiguousarray(np.concatenate(pairs).astype(np.int32))
    assert allp.shape[0] == exp["policy_shadow"]["count"]
    assert sha(allp) == exp["policy_shadow"]["sha256"]


@pytest.mark.parametrize("mod", [3, 10**9])
def test_crosscheck_group_counts(mod):
    """user_crosscheck with few groups (LDS counting sort) and with one group
    per pod (G > 8192: the atomic fallback), against M itself."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano._bits import set_bit_indices, words_to_bool
    from kano.synth import make_config
    cl = make_config("C2")
    n = cl.n
    gid = (np.arange(n) % mod).astype(np.int32)
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    r = eng.verify(gid, ngroups=int(gid.max()) + 1, shadow=False)
    M = np.stack([words_to_bool(w, n) for w in eng.rows(0, n)])   # n x n bools
    # cross[j] = exists i: M[i, j] and g(i) != g(j): column count minus the
    # count from j's own group
    total = M.sum(axis=0)
    if mod >= n:
        same = M[np.arange(n), np.arange(n)].astype(np.int64)
    else:
        per_group = np.stack([M[gid == g].sum(axis=0) for g in range(mod)])
        same = per_group[gid, np.arange(n)]
    cross = total - same > 0
    assert r["user_crosscheck"].tolist() == np.flatnonzero(cross).tolist()
    assert set_bit_indices(eng.crosscheck(gid), n).tolist() == np.flatnonzero(cross).tolist()
    eng.close()


def test_row_shards_combine_to_full():
    """Row-sharded contexts (the multi-GPU partition) reproduce the full
    matrix; their column flags combine by MAX (= OR) exactly."""
    from kano._engine import DeviceBuild
    from kano._intern import intern
    from oracle import kano_oracle as orc
    obj = cluster("s_sparse_2000")
    cs, ps = api_objects(obj)
    t = intern(cs, ps)
    n = len(cs)
    ref = orc.run_c(obj, label=obj["label"])
    from kano._intern import group_ids
    gid = group_ids(cs, obj["label"])
    cuts = [0, 333, 1000, 1001, n]
    rows, ors, nands, cross, pairs = [], [], [], [], []
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        e = DeviceBuild(t, rows=(r0, r1))
        rows.append(e.rows(r0, r1 - r0))
        ca, co = e.col_checks()
        ors.append(co)
        nands.append(~ca)
        cross.append(e.crosscheck(gid))
        pairs.append(e.shadow())
        # row classes are shard-local: select bits only for the shard's pods
        from kano._bits import words_to_bool
        cls = e.classes()
        assert (cls[:r0] == -1).all() and (cls[r1:] == -1).all() and (cls[r0:r1] >= 0).all()
        for p in (0, 7, len(ps) - 1):
            sel, _ = e.policy_sets(p)
            full = words_to_bool(ref["sel"][p], n)
            mask = np.zeros(n, bool)
            mask[r0:r1] = True
            assert np.array_equal(words_to_bool(sel, n), full & mask)
        e.close()
    assert np.array_equal(np.concatenate(rows), ref["M"])
    from kano._bits import set_bit_indices, words_to_bool
    co = np.bitwise_or.reduce(ors)
    ca = ~np.bitwise_or.reduce(nands)
    assert set_bit_indices(ca, n).tolist() == ref["all_reachable"]
    assert np.flatnonzero(~words_to_bool(co, n)).tolist() == ref["all_isolated"]
    assert set_bit_indices(np.bitwise_or.reduce(cross), n).tolist() == ref["user_crosscheck"]
    assert np.array_equal(np.concatenate(pairs), ref["shadow"])


def test_mutation_then_checks():
    """m[i, j] = v writes the device matrix; checks then see the new matrix."""
    from kano.model import ReachabilityMatrix
    from kano.algorithm import all_isolated, all_reachable, user_crosscheck, system_isolation
    from oracle import kano_oracle as orc
    obj = cluster("s_sparse_200")
    cs, ps = api_objects(obj)
    m = ReachabilityMatrix.build_matrix(cs, ps)
    n = len(cs)
    row5 = m.getrow(5)
    j = row5.index(0)
    iso_before = all_isolated(m)
    m[5, j] = 1
    assert m[5, j] == 1 and m.getrow(5)[j] == 1
    assert j not in all_isolated(m)
    assert set(all_isolated(m)) == set(iso_before) - {j}
    row = m.matrix[7]
    row.setall(1)
    assert m.getrow(7).count() == n
    M = m.engine.rows(0, n)
    from _golden import words_to_rows01
    # oracle checks over the mutated matrix
    import ctypes
    reach = np.zeros(n, np.uint8)
    isol = np.zeros(n, np.uint8)
    orc.lib().oracle_column_checks(n, orc._p(np.ascontiguousarray(M)), 0, n, orc._p(reach),
                                   orc._p(isol))
    assert all_reachable(m) == np.flatnonzero(reach).tolist()
    assert all_isolated(m) == np.flatnonzero(isol).tolist()
    gid = orc.group_ids_json(obj, obj["label"])
    cross = np.zeros(n, np.uint8)
    orc.lib().oracle_crosscheck(n, orc._p(np.ascontiguousarray(M)), orc._p(gid), 0, n,
                                orc._p(cross))
    assert user_crosscheck(m, cs, obj["label"]) == np.flatnonzero(cross).tolist()
    assert system_isolation(m, 7) == []


def test_explicit_matrix_constructor():
    from kano.model import ReachabilityMatrix, BitArray
    from kano.algorithm import all_reachable, all_isolated, system_isolation
    rows = ["110", "010", "011"]
    m = ReachabilityMatrix(3, [BitArray(r) for r in rows])
    assert [r.to01() for r in m.matrix] == rows
    assert all_reachable(m) == [1] and all_isolated(m) == [] and system_isolation(m, 1) == [0, 2]


def test_degenerate_sizes():
    from kano.model import ReachabilityMatrix, Container, Policy, PolicySelect, PolicyAllow
    from kano.model import PolicyEgress, PolicyProtocol
    from kano.algorithm import all_reachable, all_isolated, policy_shadow, policy_conflict
    m = ReachabilityMatrix.build_matrix([], [])
    assert all_reachable(m) == [] and all_isolated(m) == [] and policy_shadow(m, [], []) == []
    cs = [Container("a", {"x": "1"}), Container("b", {})]
    m = ReachabilityMatrix.build_matrix(cs, [])
    assert all_isolated(m) == [0, 1] and policy_conflict(m, [], cs) == []
    ps = [Policy("p", PolicySelect({}), PolicyAllow({}), PolicyEgress, PolicyProtocol([]))]
    m = ReachabilityMatrix.build_matrix(cs, ps)
    assert all_reachable(m) == [0, 1] and [r.to01() for r in m.matrix] == ["11", "11"]


def _mixed_cluster(seed, n=300, P=60, nkeys=6):
    """Labels of mixed Python types (ints, floats equal to ints, bools, strings,
    NaN) over a few keys, selectors drawn from the same values: the interning
    folds == classes and NaN never matches (quirk Q7)."""
    import math
    rng = np.random.default_rng(seed)
    vals = [0, 1, 2, 1.0, True, "1", "a", "b", math.nan, 3, 4.5]
    keys = [f"k{i}" for i in range(nkeys)]
    pods = []
    for i in range(n):
        labels = {}
        for k in keys:
            if rng.random() < 0.7:
                labels[k] = vals[rng.integers(len(vals))]
        labels["tenant"] = f"t{rng.integers(4)}"
        pods.append({"name": f"p{i}", "labels": labels})
    pols = []
    for p in range(P):
        sel = {k: vals[rng.integers(len(vals))]
               for k in rng.choice(keys, size=rng.integers(0, 3), replace=False)}
        alw = {k: vals[rng.integers(len(vals))]
               for k in rng.choice(keys, size=rng.integers(0, 3), replace=False)}
        pols.append({"name": f"q{p}", "select": sel, "allow": alw,
                     "direction": "ingress" if rng.random() < 0.5 else "egress",
                     "protocol": ["TCP", "80"]})
    return {"label": "tenant", "pods": pods, "policies": pols}


@pytest.mark.parametrize("packed", ["1", "0"])
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_mixed_types_packed_and_unpacked(seed, packed, monkeypatch):
    """Class hashing on packed key words (value id + 3, ids >= -3 with NaN's
    -3) and on gathered pod values give the oracle's matrix and checks."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    from kano._bits import set_bit_indices, words_to_bool
    from oracle import kano_oracle as orc
    monkeypatch.setenv("KANO_TUNE", f"packed={packed}")
    obj = _mixed_cluster(seed)
    cs, ps = api_objects(obj)
    ref = orc.run_c(obj, label="tenant")
    eng = DeviceBuild(intern(cs, ps))
    n = len(cs)
    assert np.array_equal(eng.rows(0, n), ref["M"])
    r = eng.verify(group_ids(cs, "tenant"), sys_row=0, shadow=True)
    assert r["all_reachable"].tolist() == ref["all_reachable"]
    assert r["all_isolated"].tolist() == ref["all_isolated"]
    assert r["user_crosscheck"].tolist() == ref["user_crosscheck"]
    assert r["system_isolation"].tolist() == ref["system_isolation"]
    assert np.array_equal(np.ascontiguousarray(r["pairs"]).reshape(-1, 2), ref["shadow"])
    eng.close()


@pytest.mark.parametrize("tune", ["", "async=0", "packed=0", "shr=4"])
@pytest.mark.parametrize("n,P", [(1, 0), (1, 1), (2, 3), (5, 1), (63, 7), (64, 64), (65, 9),
                                 (130, 40)])
def test_verify_small_shapes_vs_oracle(n, P, tune, monkeypatch):
    """kano_verify on tiny and word-boundary shapes (1, 63, 64, 65 pods; no
    policy; more policies than pods) with synchronous and asynchronous
    completion and both classification forms: every
    list, the pairs and the count-only count equal the C oracle's (a
    restatement of algorithm.py:4-80)."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    from kano.synth import make_cluster, objects_from_json
    from kano import model
    from oracle import kano_oracle as orc
    monkeypatch.setenv("KANO_TUNE", tune)
    obj = make_cluster(n, P, "sparse", seed=n * 1000 + P).to_json_obj()
    ref = orc.run_c(obj, label="tenant")
    cs, ps = objects_from_json(obj, model)
    gid = group_ids(cs, "tenant")
    eng = DeviceBuild(intern(cs, ps), build=False)
    for sys_row in sorted({0, n - 1}):
        r = eng.verify(gid, sys_row=sys_row, shadow=True)
        assert r["all_reachable"].tolist() == ref["all_reachable"]
        assert r["all_isolated"].tolist() == ref["all_isolated"]
        assert r["user_crosscheck"].tolist() == ref["user_crosscheck"]
        row = ref["M"][sys_row]
        bits = np.unpackbits(row.view(np.uint8), bitorder="little")[:n]
        assert r["system_isolation"].tolist() == np.flatnonzero(bits == 0).tolist()
        assert r["shadow_count"] == ref["shadow_count"]
        assert np.array_equal(np.asarray(r["pairs"]).reshape(-1, 2), ref["shadow"].reshape(-1, 2))
        assert np.array_equal(eng.rows(0, n), ref["M"])
        c = eng.verify(gid, sys_row=sys_row, shadow=True, shadow_count_only=True)
        assert c["shadow_count"] == ref["shadow_count"] and c["pairs"] is None
    eng.close()
