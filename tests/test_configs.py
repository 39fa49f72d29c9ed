"""Full-size parity: BASELINE.json's configs C3 / C4 against kano_py's own
outputs (tests/golden/expected/C3.json, C4.json from make_golden.py --big, the
reference run on the same seeded clusters), C5 (1M pods / 100k policies, out
of kano_py's and the host's reach: 125 GB) by size-independent properties,
the reference generator's clusters (kano_py/tests/generate.py, seeded, through
the YAML files and the parser as kano_py/tests/test_basic.py:16-37 does), and
the k_rows variants that only fire on wide matrices forced at small n.

All of it goes through the C ABI: kano_verify (the bench's step), the matrix
rows, the class-level lists expanded to Container.select_policies /
allow_policies, and the policies' working sets."""
import hashlib
import os
import sys

import numpy as np
import pytest

from _golden import (GOLDEN, allow_lists_csr, cluster, container_lists_csr, csr_sha, expected,
                     index_list_matches, row_digest, sha)

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(GOLDEN))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from kano import _native
    if not _native.gpu_available():
        pytest.fail("GPU test run without a usable HIP device / libkano_hip.so")


def tenant_groups(cl):
    from kano.synth import KEY_NAMES
    return np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)


def check_verify(r, exp, shadow=True):
    """kano_verify's result lists against kano_py's (algorithm.py:4-80)."""
    assert index_list_matches(r["all_reachable"], exp["all_reachable"])
    assert index_list_matches(r["all_isolated"], exp["all_isolated"])
    assert index_list_matches(r["user_crosscheck"], exp["user_crosscheck"]["result"])
    assert index_list_matches(r["system_isolation"], exp["system_isolation"]["result"])
    if shadow:
        assert r["shadow_count"] == exp["policy_shadow"]["count"]
        assert sha(np.ascontiguousarray(r["pairs"], dtype=np.int32)) == \
            exp["policy_shadow"]["sha256"]


def check_build(eng, exp, n, P):
    """M rows, Container.select_policies / allow_policies and the policies'
    working sets (model.py:125-165) against kano_py's hashes."""
    M = eng.rows(0, n)
    assert sha(M) == exp["M_sha256"]
    del M
    cls = eng.classes()
    so, sp = eng.select_csr()
    assert csr_sha(*container_lists_csr(cls, so, sp)) == exp["select_policies_sha256"]
    ao, ap = eng.allow_csr()
    assert csr_sha(*allow_lists_csr(n, ao, ap)) == exp["allow_policies_sha256"]
    W = (n + 63) // 64
    S = np.zeros((P, W), np.uint64)
    A = np.zeros((P, W), np.uint64)
    for p in range(P):
        S[p], A[p] = eng.policy_sets(p)
    assert sha(S) == exp["sel_sha256"]
    assert sha(A) == exp["allow_sha256"]


@pytest.mark.parametrize("name", ["C3", "C4"])
def test_config_vs_kano_py(name):
    """C3 (sparse, the headline config) and C4 (broad selectors, the dense
    path) bit-exact against kano_py through the bench's step.  C4's
    policy_shadow (~1e11 tuples) is checked as a count (count-only mode)
    against the C oracle's count (kano_py cannot hold the list)."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_config
    exp = expected(name)
    cl = make_config(name)
    assert cl.fingerprint() == exp["seed"]["fingerprint"]
    n, P = cl.n, cl.P
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    eng.set_groups(tenant_groups(cl))
    full_shadow = "sha256" in exp["policy_shadow"]
    if full_shadow:
        r = eng.verify("stored", sys_row=0, shadow=True)
        check_verify(r, exp)
        r = eng.verify("stored", sys_row=0, shadow=True, shadow_count_only=True)
        assert r["shadow_count"] == exp["policy_shadow"]["count"]
    else:
        r = eng.verify("stored", sys_row=0, shadow=True, shadow_count_only=True)
        check_verify(r, exp, shadow=False)
        assert r["shadow_count"] == exp["policy_shadow"]["oracle_count"]
    check_build(eng, exp, n, P)
    if name == "C4":   # the dense path, forced both ways
        for path in ("bitwise", "mfma"):
            r = eng.verify("stored", sys_row=0, shadow=False, path=path)
            check_verify(r, exp, shadow=False)
            assert sha(eng.rows(0, n)) == exp["M_sha256"]
    eng.close()


# --- C5: 1M pods / 100k policies (125 GB) by properties ----------------------
def _select_policies_host(tb, i):
    """Policies whose working selector matches pod i (model.py:95-111 on
    the interned ids: every kept term (col, val) must equal the pod's value;
    unknown keys were dropped at interning, quirk Q1)."""
    off, col, val = tb.sel_off, tb.sel_col, tb.sel_val
    ok = tb.pod_val[col, i] == val
    bad = np.zeros(tb.P, np.int64)
    np.add.at(bad, np.repeat(np.arange(tb.P), np.diff(off)), ~ok)
    return np.flatnonzero(bad == 0)


def _allow_set_host(tb, p):
    """allow_p over all pods, the same predicate on the allow side."""
    a0, a1 = tb.alw_off[p], tb.alw_off[p + 1]
    m = np.ones(tb.n, bool)
    for t in range(a0, a1):
        m &= tb.pod_val[tb.alw_col[t]] == tb.alw_val[t]
    return m


def _pack(bits):
    n = bits.shape[0]
    W = (n + 63) // 64
    buf = np.zeros(W * 64, np.uint8)
    buf[:n] = bits
    return np.packbits(buf, bitorder="little").view("<u8")


def test_c5_full_size_properties():
    """C5 at full size on one GPU: (0) every check list, policy_shadow's
    pairs (count + sha256) and the digest of all 10^6 rows equal C5's record
    (tests/golden/make_c5.py: oracle/kano_indexed.py, pinned on C2-C4 against
    kano_py, tests/test_oracle_indexed.py); (1) sampled rows -- the largest row
    classes' first members, row 0, the last row and random rows -- equal
    OR_{p: sel_p[i]} allow_p recomputed on the host from the tables
    (model.py:158-160); the device digest of each equals the host digest
    of the fetched row; (2) the bitwise and MFMA paths give the same row
    digests; (3) 8 row shards (the multi-GPU partition) give the same row
    digests and, through kano_verify_shard / kano_verify_combine, the same
    column lists as the unsharded step."""
    import torch
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_config
    cl = make_config("C5")
    tb = tables_from_cluster(cl)
    n = cl.n
    gid = tenant_groups(cl)
    eng = DeviceBuild(tb, build=False)
    eng.set_groups(gid)
    full = eng.verify("stored", sys_row=0, shadow=True)
    full = {k: (np.array(v, copy=True) if v is not None else None) for k, v in full.items()}
    dig = eng.rows_digest(0, n)
    # (0) the independent record
    exp = expected("C5")
    assert exp["seed"]["fingerprint"] == cl.fingerprint()
    check_verify(full, exp)
    assert hashlib.sha256(np.ascontiguousarray(dig, dtype="<u8").tobytes()).hexdigest() == \
        exp["row_digests_sha256"]
    smp = exp["row_digest_sample"]
    assert [f"{int(d):016x}" for d in dig[smp["rows"]]] == smp["digest"]
    # (1) sampled rows against the host restatement
    cls = eng.classes()
    big = np.argsort(-np.bincount(cls))[:24]
    first = np.full(cls.max() + 1, -1, np.int64)
    first[cls[::-1]] = np.arange(n - 1, -1, -1)
    rng = np.random.default_rng(5)
    sample = np.unique(np.concatenate([first[big], [0, n - 1], rng.integers(0, n, 40)]))
    cache = {}
    for i in sample:
        row = eng.rows(int(i), 1)[0]
        assert row_digest(row)[0] == dig[i]
        acc = np.zeros(n, bool)
        for p in _select_policies_host(tb, int(i)):
            if p not in cache:
                cache[p] = _allow_set_host(tb, int(p))
            acc |= cache[p]
        assert np.array_equal(row, _pack(acc)), f"row {i}"
    # system_isolation(0) is row 0's zeros
    row0 = eng.rows(0, 1)[0]
    bits0 = np.unpackbits(row0.view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(full["system_isolation"], np.flatnonzero(bits0 == 0))
    # (2) the MFMA contraction path writes the same rows
    eng.verify("stored", sys_row=0, shadow=False, path="mfma")
    assert np.array_equal(eng.rows_digest(0, n), dig)
    eng.close()
    # (3) 8 row shards, one after the other on this device
    N = 8
    W = (n + 63) // 64
    gathered = torch.zeros(N * 3 * W, dtype=torch.int64, device="cuda")
    spans = [(k * n // N, (k + 1) * n // N) for k in range(N)]
    shadow_total = 0
    pairs = []
    for k, (r0, r1) in enumerate(spans):
        e = DeviceBuild(tb, rows=(r0, r1), build=False)
        e.verify_shard(gathered.data_ptr() + 8 * 3 * W * k, gid=gid, sys_row=0, shadow=True)
        torch.cuda.synchronize()
        if k == N - 1:
            # every shard's words are in: the combine on the last shard
            r = e.verify_combine(gathered.data_ptr(), N)
            for key in ("all_reachable", "all_isolated", "user_crosscheck"):
                assert np.array_equal(r[key], full[key]), key
            shadow_total += r["shadow_count"]
            pairs.append(np.array(r["pairs"], copy=True))
        else:
            r = e.verify_combine(gathered.data_ptr(), N)   # partial: only the shard's own
            shadow_total += r["shadow_count"]
            pairs.append(np.array(r["pairs"], copy=True))
        # (the shard's rows are written by the combine half)
        assert np.array_equal(e.rows_digest(r0, r1 - r0), dig[r0:r1]), f"shard {k}"
        e.close()
    assert shadow_total == full["shadow_count"]
    assert np.array_equal(np.concatenate(pairs), full["pairs"])


@pytest.mark.parametrize("N", [2, 4, 8])
def test_c3_row_shards_vs_kano_py(N):
    """C3 -- the headline config the metric quotes at 1/2/4/8 GPUs -- as N row
    shards (kano/shard.py row_range, the multi-GPU partition), every shard
    alive at once on this device: each shard's kano_verify_shard writes its
    column words into one gathered buffer (what the all-gather delivers), then
    every shard's kano_verify_combine must give kano_py's all_reachable,
    all_isolated and user_crosscheck lists (algorithm.py:4-42), the owner of
    row 0 its system_isolation list (algorithm.py:45-55); the shards' rows
    concatenated in rank order hash to kano_py's M (model.py:158-160), and
    their policy_shadow pairs concatenated in rank order equal kano_py's list
    (algorithm.py:58-80: per pod in row order)."""
    import torch
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.shard import row_range
    from kano.synth import make_config
    cl = make_config("C3")
    exp = expected("C3")
    assert cl.fingerprint() == exp["seed"]["fingerprint"]
    tb = tables_from_cluster(cl)
    gid = tenant_groups(cl)
    n = cl.n
    W = (n + 63) // 64
    gathered = torch.zeros(N * 3 * W, dtype=torch.int64, device="cuda")
    spans = [row_range(n, N, k) for k in range(N)]
    engs = []
    try:
        for k, (r0, r1) in enumerate(spans):
            e = DeviceBuild(tb, rows=(r0, r1), build=False)
            engs.append(e)
            e.verify_shard(gathered.data_ptr() + 8 * 3 * W * k, gid=gid, sys_row=0, shadow=True)
        torch.cuda.synchronize()   # every shard's words are in (the all-gather's end)
        h = hashlib.sha256()
        pairs, total = [], 0
        for k, (e, (r0, r1)) in enumerate(zip(engs, spans)):
            r = e.verify_combine(gathered.data_ptr(), N)
            for key in ("all_reachable", "all_isolated"):
                assert index_list_matches(r[key], exp[key]), (N, k, key)
            assert index_list_matches(r["user_crosscheck"], exp["user_crosscheck"]["result"]), \
                (N, k)
            if r0 == 0:
                assert index_list_matches(r["system_isolation"],
                                          exp["system_isolation"]["result"]), (N, k)
            else:
                assert r["system_isolation"] is None
            total += r["shadow_count"]
            pairs.append(np.array(r["pairs"], copy=True))
            h.update(np.ascontiguousarray(e.rows(r0, r1 - r0)).tobytes())
        assert h.hexdigest() == exp["M_sha256"]
        assert total == exp["policy_shadow"]["count"]
        allp = np.ascontiguousarray(np.concatenate(pairs), dtype=np.int32)
        assert sha(allp) == exp["policy_shadow"]["sha256"]
    finally:
        for e in engs:
            e.close()


# --- D1: the dense path (MFMA GEMM) at full size ----------------------------
def test_d1_dense_auto_picks_mfma():
    """D1 (kano/synth.py dense mode: 8,000 row classes, each selected by
    ~2,250 of 10^4 policies): AUTO takes the int8 MFMA GEMM for the heavy
    classes, and kano_verify's lists, policy_shadow's count (every subset
    test; the pairs would be ~5e11) and the digest of every row equal D1's record (tests/golden/make_c5.py,
    oracle/kano_indexed.py); the bitwise OR writes the same rows."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_config
    cl = make_config("D1")
    exp = expected("D1")
    assert exp["seed"]["fingerprint"] == cl.fingerprint()
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    eng.set_groups(tenant_groups(cl))
    r = eng.verify("stored", sys_row=0, shadow=True, shadow_count_only=True)
    info = eng.info()
    assert info["HEAVY_PATH"] == 2 and info["HEAVY_KERNEL"] == 3, info   # the MFMA GEMM
    assert info["HEAVY"] >= 4096, info
    check_verify(r, exp, shadow=False)
    assert r["shadow_count"] == exp["policy_shadow"]["count"]   # ~5e11 pairs: the count
    dig = eng.rows_digest(0, cl.n)
    assert hashlib.sha256(np.ascontiguousarray(dig, dtype="<u8").tobytes()).hexdigest() == \
        exp["row_digests_sha256"]
    eng.verify("stored", sys_row=0, shadow=False, path="bitwise")
    assert eng.info()["HEAVY_PATH"] == 1
    assert np.array_equal(eng.rows_digest(0, cl.n), dig)
    eng.close()


def test_d1_vs_kano_py():
    """D1 bit-exact against kano_py itself (tests/golden/expected/
    D1_kano_py.json, make_golden.py --big D1: kano_py's build_matrix and
    checks on the same seeded cluster, ~2 h on one core): the matrix, both
    list CSRs, the policies' working sets and the four index lists, through
    the bench's step with the MFMA GEMM chosen.  policy_shadow (~5e11 pairs)
    is beyond kano_py's list: its count stays pinned by D1.json (the indexed
    restatement, whose count-only branch equals kano_py's counts on C2 / C3,
    tests/test_oracle_indexed.py)."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_config
    if not os.path.exists(os.path.join(GOLDEN, "expected", "D1_kano_py.json")):
        pytest.skip("no kano_py record of D1")
    cl = make_config("D1")
    exp = expected("D1_kano_py")
    assert exp["seed"]["fingerprint"] == cl.fingerprint()
    eng = DeviceBuild(tables_from_cluster(cl), build=False)
    eng.set_groups(tenant_groups(cl))
    r = eng.verify("stored", sys_row=0, shadow=True, shadow_count_only=True)
    info = eng.info()
    assert info["HEAVY_PATH"] == 2 and info["HEAVY_KERNEL"] == 3, info   # the MFMA GEMM
    check_verify(r, exp, shadow=False)
    assert r["shadow_count"] == expected("D1")["policy_shadow"]["count"]
    check_build(eng, exp, cl.n, cl.P)
    eng.close()


# --- the reference generator's clusters (kano_py/tests/generate.py) ----------
GEN_NAMES = sorted(f[:-5] for f in os.listdir(os.path.join(GOLDEN, "expected"))
                   if f.startswith("gen_"))


def gen_objects(exp, tmp_path):
    """generate.py's pods and YAML files (seeded restatement, refgen.py),
    the files parsed by the drop-in parser in the order kano_py's walk
    visited them (kano_py/tests/test_basic.py:16-22)."""
    from refgen import RefGen
    from kano import model
    from kano.parser import ConfigParser
    g = exp["generator"]
    rg = RefGen(g["seed"], podN=g["podN"], policyN=g["policyN"])
    assert rg.digest() == g["digest"]
    rg.write(str(tmp_path))
    cp = ConfigParser()
    for f in exp["walk_order"]:
        cp.parse(str(tmp_path / f))
    assert len(cp.policies) == exp["P"]
    cs = [model.Container(name, labels) for name, labels in rg.pods]
    return cs, cp.policies


@pytest.mark.parametrize("name", GEN_NAMES)
def test_reference_generator_clusters(name, tmp_path):
    """generate -> YAML -> ConfigParser -> build_matrix -> checks, bit-exact
    against kano_py on the same files; up to density 1.0 (gen_s6_20000) and
    5M shadow pairs.  Small ones through the drop-in API, all through
    kano_verify."""
    from kano.model import ReachabilityMatrix
    from kano import algorithm as alg
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    exp = expected(name)
    cs, ps = gen_objects(exp, tmp_path)
    n = len(cs)
    if n <= 4000:
        m = ReachabilityMatrix.build_matrix(cs, ps)
        assert sha(m.engine.rows(0, n)) == exp["M_sha256"]
        assert index_list_matches(alg.all_reachable(m), exp["all_reachable"])
        assert index_list_matches(alg.all_isolated(m), exp["all_isolated"])
        assert index_list_matches(alg.user_crosscheck(m, cs, "User"),
                                  exp["user_crosscheck"]["result"])
        pairs = alg.policy_shadow(m, ps, cs)
        assert len(pairs) == exp["policy_shadow"]["count"]
        assert sha(np.array(pairs, np.int32).reshape(-1, 2)) == exp["policy_shadow"]["sha256"]
        assert csr_sha(*_lists(cs, "select")) == exp["select_policies_sha256"]
        assert csr_sha(*_lists(cs, "allow")) == exp["allow_policies_sha256"]
    eng = DeviceBuild(intern(cs, ps), build=False)
    r = eng.verify(group_ids(cs, "User"), sys_row=0, shadow=True)
    check_verify(r, exp)
    check_build(eng, exp, n, len(ps))
    eng.close()


def _lists(cs, which):
    from _golden import lists_to_csr
    return lists_to_csr([c.select_policies if which == "select" else c.allow_policies
                         for c in cs])


# --- matrix-write forms ------------------------------------------------------
@pytest.mark.parametrize("tune", ["", "cww=64", "cww=16", "async=0",
                                  "hexplds=3", "hexplds=4", "dx=2", "aclds=0", "rch=3",
                                  "rch=64,cww=16384", "shr=4", "shr=8", "rw=2", "rw=2,rch=1",
                                  "rw=2,cww=16", "rw=2,rch=64,async=0", "rw=2,rwg=3",
                                  "rw=2,rwg=1,rch=1", "sww=1", "sww=3", "aipt=8", "aipt=3", "rheavy=0", "rheavy=1"])
@pytest.mark.parametrize("name", ["C2", "s_sparse_2000", "s_broad_1000", "q_wide_select"])
def test_rows_variants_forced(name, tune, monkeypatch):
    """The matrix write's shipped forms -- k_rows and the persistent k_rows_w,
    the heavy rows' forms, the column chunks wide matrices take (forced at
    small n), with and without asynchronous completion -- against kano_py's
    matrix and lists."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids, tables_from_cluster
    from kano.synth import make_config, objects_from_json
    from kano import model
    monkeypatch.setenv("KANO_TUNE", tune)
    exp = expected(name)
    if name == "C2":
        cl = make_config("C2")
        t = tables_from_cluster(cl)
        gid = tenant_groups(cl)
    else:
        obj = cluster(name)
        cs, ps = objects_from_json(obj, model)
        t = intern(cs, ps)
        gid = group_ids(cs, obj.get("label", "app"))
    eng = DeviceBuild(t, build=False)
    r = eng.verify(gid, sys_row=0, shadow=True)
    check_verify(r, exp)
    assert sha(eng.rows(0, t.n)) == exp["M_sha256"]
    assert eng.info()["ROWS_KERNEL"] in (2, 3, 4, 5, 6)
    # the bench's form: page-locked result buffers (the whole tail queued at
    # once, sized on the device), twice back to back
    from kano._engine import PinnedBuffer
    pi, pp = PinnedBuffer(16 * max(t.n, 1)), PinnedBuffer(8 << 20)
    for _ in range(2):
        r = eng.verify(gid, sys_row=0, shadow=True, idx=pi.view(np.int32, 4 * max(t.n, 1)),
                       pairs=pp.view(np.int32, 2 << 20))
        check_verify(r, exp)
    assert sha(eng.rows(0, t.n)) == exp["M_sha256"]
    eng.build()
    assert sha(eng.rows(0, t.n)) == exp["M_sha256"]
    eng.close()


# --- policy_shadow's count without the pairs --------------------------------
@pytest.mark.parametrize("mode", ["shcount=0", "shcount=1", "shcount=2", "shcount=2,shgsub=0",
                                  "shcount=1,shr=4", "shcount=1,shr=8"])
@pytest.mark.parametrize("name", ["C2", "s_broad_1000", "s_broad_300", "s_sparse_2000", "q_shadow",
                                  "q_wide_select", "gen_s5_10000", "gen_s4_4000"])
def test_shadow_count_only_vs_kano_py(name, mode, tmp_path, monkeypatch):
    """kano_verify's count-only policy_shadow -- the pairwise subset tests
    without the flags (shcount=1), the policies grouped by allow set with one
    subset test per pair of groups (shcount=2), or the automatic choice --
    equals len(policy_shadow(...)) as kano_py computed it, whole and summed
    over row shards."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids, tables_from_cluster
    from kano.synth import make_config, objects_from_json
    from kano import model
    monkeypatch.setenv("KANO_TUNE", mode)
    exp = expected(name)
    if name == "C2":
        t = tables_from_cluster(make_config("C2"))
    elif name.startswith("gen_"):
        cs, ps = gen_objects(exp, tmp_path)
        t = intern(cs, ps)
    else:
        cs, ps = objects_from_json(cluster(name), model)
        t = intern(cs, ps)
    eng = DeviceBuild(t, build=False)
    r = eng.verify(None, sys_row=0, shadow=True, shadow_count_only=True)
    assert r["shadow_count"] == exp["policy_shadow"]["count"]
    assert r["pairs"] is None
    assert index_list_matches(r["all_isolated"], exp["all_isolated"])
    eng.close()
    n = t.n
    total = 0
    for r0, r1 in [(0, n // 3), (n // 3, n)]:
        e = DeviceBuild(t, rows=(r0, r1), build=False)
        total += e.verify(None, sys_row=0, shadow=True, shadow_count_only=True)["shadow_count"]
        e.close()
    assert total == exp["policy_shadow"]["count"]
