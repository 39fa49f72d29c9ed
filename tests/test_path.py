"""Multi-hop reachability: kubesv's `path` relation
(kubesv/kubesv/constraint.py:233-237) over kano's matrix.

kubesv runs on z3 (not installed), so the composition rule is restated twice
(oracle/kano_oracle.c oracle_path, and the Datalog rules on Python sets,
kano_oracle.path_py) and applied to matrices pinned by kano_py's golden
vectors; the GPU path (libkano_hip.so kano_path) must equal it bit for bit."""
import numpy as np
import pytest

from _golden import cluster, expected, rows01_to_words, sha


def _rand_words(n, density, seed):
    rng = np.random.default_rng(seed)
    B = rng.random((n, n)) < density
    W = (n + 63) // 64
    pad = np.zeros((n, W * 64), bool)
    pad[:, :n] = B
    return B, np.packbits(pad, axis=1, bitorder="little").view("<u8").reshape(n, W)


@pytest.mark.parametrize("n,density", [(1, 1.0), (5, 0.3), (70, 0.03), (130, 0.01), (200, 0.2)])
@pytest.mark.parametrize("hops", [1, 2, 3, 0])
def test_oracle_path_matches_rules(n, density, hops):
    """oracle_path == the Datalog rules on sets == numpy boolean products."""
    from oracle import kano_oracle as orc
    B, M = _rand_words(n, density, n * 7 + hops)
    P, _ = orc.path_c(M, n, hops)
    got = {(i, j) for i in range(n) for j in range(n) if (int(P[i, j >> 6]) >> (j & 63)) & 1}
    edges = {(int(i), int(j)) for i, j in zip(*np.nonzero(B))}
    assert got == orc.path_py(edges, n, hops)
    R = B.copy()
    k = 1
    while hops == 0 or k < hops:
        Rn = R | ((R.astype(np.int64) @ B.astype(np.int64)) > 0)
        k += 1
        if (Rn == R).all():
            break
        R = Rn
    assert got == {(int(i), int(j)) for i, j in zip(*np.nonzero(R))}


def test_oracle_path_paper_example():
    """Known answers on kano_py's paper example (SURVEY §A.5 matrix)."""
    from oracle import kano_oracle as orc
    rows = ["11010", "10010", "10010", "01000", "00100"]
    M = rows01_to_words(rows, 5)
    P2, _ = orc.path_c(M, 5, 2)
    Pc, _ = orc.path_c(M, 5, 0)
    from _golden import words_to_rows01
    assert words_to_rows01(P2, 5) == ["11010", "11010", "11010", "11010", "10110"]
    assert words_to_rows01(Pc, 5) == ["11010", "11010", "11010", "11010", "11110"]


# ---------------------------------------------------------------------------
# GPU parity
PATH_CLUSTERS = ["q_dirs", "q_shadow", "q_unknown_key", "s_sparse_50", "s_sparse_500",
                 "s_sparse_2000", "s_broad_300", "s_broad_1000"]


def _built(name):
    from kano import model
    from kano.synth import objects_from_json
    cs, ps = objects_from_json(cluster(name), model)
    return model.ReachabilityMatrix.build_matrix(cs, ps), cs, ps


@pytest.mark.gpu
@pytest.mark.parametrize("name", PATH_CLUSTERS)
@pytest.mark.parametrize("hops", [2, 3, 0])
@pytest.mark.parametrize("mode", ["auto", "bitwise", "mfma"])
def test_path_matches_oracle(name, hops, mode):
    from kano import algorithm as alg
    from oracle import kano_oracle as orc
    m, cs, ps = _built(name)
    n = m.container_size
    M = m.engine.rows(0, n)
    # the matrix the path starts from is kano_py's (pinned)
    from _golden import sha
    assert sha(M) == expected(name)["M_sha256"]
    ref, _ = orc.path_c(M, n, hops)
    pm = alg.transitive_closure(m, mode) if hops == 0 else alg.k_hop(m, hops, mode)
    assert np.array_equal(pm.engine.rows(0, n), ref)
    if mode == "mfma" and pm.path_info["steps_run"] > 0:
        assert pm.path_info["mfma_steps"] == pm.path_info["steps_run"]
    if mode == "bitwise":
        assert pm.path_info["mfma_steps"] == 0
    # every query reads the path matrix
    col_or = np.bitwise_or.reduce(ref, axis=0) if n else None
    iso = [j for j in range(n) if not (int(col_or[j >> 6]) >> (j & 63)) & 1]
    assert alg.all_isolated(pm) == iso
    assert alg.system_isolation(pm, 0) == [
        j for j in range(n) if not (int(ref[0, j >> 6]) >> (j & 63)) & 1]


@pytest.mark.gpu
def test_two_hop_paper_example():
    from kano import algorithm as alg
    from kano.model import ReachabilityMatrix
    from sample import paper_example
    cs, ps = paper_example()
    m = ReachabilityMatrix.build_matrix(cs, ps)
    p2 = alg.two_hop(m)
    assert [[p2[i, j] for j in range(5)] for i in range(5)] == [
        [1, 1, 0, 1, 0], [1, 1, 0, 1, 0], [1, 1, 0, 1, 0], [1, 1, 0, 1, 0], [1, 0, 1, 1, 0]]
    pc = alg.transitive_closure(m)
    assert pc.getrow(4).tolist() == [1, 1, 1, 1, 0]
    assert alg.all_isolated(pc) == [4]
    # the source matrix is untouched
    assert m.getrow(4).tolist() == [0, 0, 1, 0, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["bitwise", "mfma"])
def test_path_edited_and_explicit_matrix(mode):
    """After an edit of M (and for an explicit matrix) the classes no longer
    describe it: the path runs on identity classes."""
    from kano import algorithm as alg
    from kano.model import ReachabilityMatrix
    from oracle import kano_oracle as orc
    m, cs, ps = _built("s_sparse_500")
    n = m.container_size
    m[3, 7] = 1
    m[7, 11] = 1
    m[0, 0] = 0
    M = m.engine.rows(0, n)
    for hops in (2, 0):
        pm = alg.k_hop(m, hops, mode) if hops else alg.transitive_closure(m, mode)
        assert pm.path_info["identity"] == 1
        assert np.array_equal(pm.engine.rows(0, n), orc.path_c(M, n, hops)[0])
    B, W = _rand_words(300, 0.004, 11)
    from kano.model import BitArray
    em = ReachabilityMatrix(300, [BitArray.from_words(W[i], 300) for i in range(300)])
    pe = alg.transitive_closure(em, mode)
    assert np.array_equal(pe.engine.rows(0, 300), orc.path_c(W, 300, 0)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [101, 102, 103])
def test_path_synthetic_seeds(seed):
    """Seeded synthetic clusters (SURVEY §8(d) generator): every mode agrees
    with the oracle on the closure and the two-hop matrix."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_cluster
    from oracle import kano_oracle as orc
    cl = make_cluster(1500, 150, "sparse" if seed != 103 else "broad", seed=seed)
    eng = DeviceBuild(tables_from_cluster(cl))
    n = cl.n
    M = eng.rows(0, n)
    for hops in (2, 0):
        ref, _ = orc.path_c(M, n, hops)
        for mode in ("auto", "bitwise", "mfma"):
            dst = DeviceBuild.empty(n)
            dst.path_from(eng, hops, mode)
            assert np.array_equal(dst.rows(0, n), ref), (hops, mode)
            dst.close()
    eng.close()


@pytest.mark.gpu
def test_path_expand_table_from_l2(monkeypatch):
    """The expansion's L2-read variant (column-class tables too large for LDS,
    forced here with KANO_TUNE=pathlds=0) writes the same matrix."""
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_cluster
    from oracle import kano_oracle as orc
    cl = make_cluster(1200, 120, "sparse", seed=105)
    eng = DeviceBuild(tables_from_cluster(cl))
    monkeypatch.setenv("KANO_TUNE", "pathlds=0")
    dst = DeviceBuild.empty(cl.n)
    dst.path_from(eng, 2, "bitwise")
    M = eng.rows(0, cl.n)
    assert np.array_equal(dst.rows(0, cl.n), orc.path_c(M, cl.n, 2)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("spans", [[(0, 700), (700, 1500)], [(0, 0), (0, 1), (1, 900), (900, 1500)]])
@pytest.mark.parametrize("hops", [2, 0])
def test_path_row_shards(spans, hops):
    """The multi-GPU path on one device: every shard writes its part of T into
    its slot of one gathered buffer (what the RCCL all-gather builds), then
    kano_path_combine writes the shard's rows; the rows concatenate to the
    single-device path matrix."""
    import torch
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_cluster
    from oracle import kano_oracle as orc
    cl = make_cluster(1500, 150, "sparse", seed=107)
    t = tables_from_cluster(cl)
    n = cl.n
    full = DeviceBuild(t)
    ref, _ = orc.path_c(full.rows(0, n), n, hops)
    engs = [DeviceBuild(t, rows=s) for s in spans]
    nw = engs[0].path_shard_words()
    assert all(e.path_shard_words() == nw for e in engs)   # column classes agree
    gathered = torch.zeros(len(spans) * max(nw, 1), dtype=torch.int64, device="cuda")
    for k, e in enumerate(engs):
        e.path_shard(gathered.data_ptr() + 8 * nw * k)
    torch.cuda.synchronize()
    rows = []
    for e, (r0, r1) in zip(engs, spans):
        dst = DeviceBuild.empty(n, rows=(r0, r1))
        dst.path_combine(e, gathered.data_ptr(), len(spans), hops, "auto")
        if r1 > r0:
            rows.append(dst.rows(r0, r1 - r0))
        dst.close()
        e.close()
    assert np.array_equal(np.concatenate(rows), ref)


@pytest.mark.gpu
def test_path_c2_scale():
    """C2 (10k pods / 1k policies, BASELINE configs[1]): the two-hop matrix
    against the oracle; the closure through size-independent properties --
    every mode gives the same matrix, it contains the two-hop matrix, and it is
    closed (the closure of the closure is itself)."""
    from kano import algorithm as alg
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.model import ReachabilityMatrix
    from kano.synth import make_config
    from oracle import kano_oracle as orc
    cl = make_config("C2")
    n = cl.n
    eng = DeviceBuild(tables_from_cluster(cl))
    m = ReachabilityMatrix.__new__(ReachabilityMatrix)
    m.container_size, m._engine = n, eng
    m._containers = m._policies = m._lists = None
    m._ncontainers = n
    M = eng.rows(0, n)
    p2 = alg.two_hop(m)
    P2 = p2.engine.rows(0, n)
    assert np.array_equal(P2, orc.path_c(M, n, 2)[0])
    closures = [alg.transitive_closure(m, mode).engine.rows(0, n)
                for mode in ("auto", "bitwise", "mfma")]
    C = closures[0]
    assert all(np.array_equal(C, x) for x in closures[1:])
    assert np.array_equal(C | P2, C)
    # closed: one more composition adds nothing (the closure of C as a matrix)
    dst = DeviceBuild.empty(n)
    dst.put_rows(0, C)
    again = DeviceBuild.empty(n)
    again.path_from(dst, 0, "auto")
    assert np.array_equal(again.rows(0, n), C)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["s_sparse_2000", "q_wide_select", "paper_example"])
def test_entry_points_after_verify(name):
    """Repeated kano_verify calls (asynchronous completion, the input sets
    alternating), then the entry points that read the build's class-level
    matrix Mc on the same context -- the standalone crosscheck, the path's
    one-hop table -- agree with the oracle, and a verify after them too."""
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    from kano import model
    from kano.synth import objects_from_json
    from kano._bits import set_bit_indices
    from oracle import kano_oracle as orc
    if name == "paper_example":
        from sample import paper_example
        cs, ps = paper_example()
        label = "app"
    else:
        cs, ps = objects_from_json(cluster(name), model)
        label = expected(name)["label"]
    eng = DeviceBuild(intern(cs, ps), build=False)
    n = eng.n
    gid = group_ids(cs, label)
    exp = expected(name)
    for _ in range(3):
        r = eng.verify(gid, sys_row=0, shadow=True)
        assert r["user_crosscheck"].tolist() == exp["user_crosscheck"]["result"]
        assert r["all_isolated"].tolist() == exp["all_isolated"]
        assert r["system_isolation"].tolist() == exp["system_isolation"]["result"]
    M = eng.rows(0, n)
    assert sha(M) == exp["M_sha256"]
    # Mc-based entry points on the same context
    assert set_bit_indices(eng.crosscheck(gid), n).tolist() == exp["user_crosscheck"]["result"]
    ref, _ = orc.path_c(M, n, 2)
    dst = DeviceBuild.empty(n)
    dst.path_from(eng, 2, "bitwise")
    assert np.array_equal(dst.rows(0, n), ref)
    # and a verify again after them
    r = eng.verify(gid, sys_row=n - 1, shadow=True)
    assert r["all_reachable"].tolist() == exp["all_reachable"]
    dst.close()
    eng.close()
