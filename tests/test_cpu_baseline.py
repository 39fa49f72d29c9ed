"""The CPU baseline of bench.py (oracle/kano_cpu.c: kano_py's algorithm on
the host's cores, OpenMP) equals kano_py's record of the cluster (C2, whole)
and the single-threaded oracle on seeded clusters: it is timed as the
reference's CPU path, so it must compute the reference's results."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-verification_amd"))


@pytest.fixture(scope="module")
def bench():
    import subprocess
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    import bench as b
    return b


@pytest.mark.parametrize("threads", [1, 3])
def test_cpu_baseline_c2_matches_kano_py(bench, threads):
    from kano.synth import make_config, KEY_NAMES
    bench._cpu_lib().cpu_threads(threads)
    cl = make_config("C2")
    gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
    r = bench.cpu_baseline(cl, gid, "C2")
    assert r["verified"] is True, r
    assert r["cores"] == threads


@pytest.mark.parametrize("seed", [3, 4])
def test_cpu_port_matches_oracle(bench, seed):
    """Matrix, lists and shadow pairs of the OpenMP port against the
    one-for-one restatement (oracle/kano_oracle.c) on seeded clusters."""
    import ctypes
    from kano.synth import make_cluster
    from oracle import kano_oracle as orc
    L = bench._cpu_lib()
    L.cpu_threads(4)
    cl = make_cluster(700, 90, "sparse", seed=seed)
    ref = orc.run_c(cl.to_json_obj(), label="tenant")
    n, P = cl.n, cl.P
    W = (n + 63) // 64
    present = cl.vals >= 0
    cnt = present.sum(axis=0)
    lab_off = np.zeros(n + 1, np.int64)
    np.cumsum(cnt, out=lab_off[1:])
    order = np.argsort(~present.T, axis=1, kind="stable")
    lab_key = np.concatenate([order[i, :cnt[i]] for i in range(n)]).astype(np.int32)
    lab_val = (cl.vals[lab_key, np.repeat(np.arange(n), cnt)].astype(np.int64)
               + lab_key.astype(np.int64) * 10_000_000)
    (so, sk, sv), (ao, ak, av) = cl.working_terms()
    sv2 = sv.astype(np.int64) + sk.astype(np.int64) * 10_000_000
    av2 = av.astype(np.int64) + ak.astype(np.int64) * 10_000_000
    allv = np.unique(np.concatenate([lab_val, sv2, av2]))
    lab_val = np.searchsorted(allv, lab_val).astype(np.int32)
    sv2 = np.searchsorted(allv, sv2).astype(np.int32)
    av2 = np.searchsorted(allv, av2).astype(np.int32)
    arrs = [np.ascontiguousarray(a, d) for a, d in ((so, np.int64), (sk, np.int32), (ao, np.int64),
                                                     (ak, np.int32))]
    so, sk, ao, ak = arrs
    M = np.empty(n * W, np.uint64)
    sel = np.empty(P * W, np.uint64)
    alw = np.empty(P * W, np.uint64)
    p = lambda a: a.ctypes.data  # noqa: E731
    L.cpu_build(n, cl.vals.shape[0], p(lab_off), p(lab_key), p(lab_val), P, p(so), p(sk), p(sv2),
                p(ao), p(ak), p(av2), p(M), p(sel), p(alw))
    assert np.array_equal(M.reshape(n, W), ref["M"])
    flags = np.empty(n, np.uint8)
    L.cpu_col_reduce(n, p(M), 0, p(flags))
    assert np.flatnonzero(flags).tolist() == ref["all_reachable"]
    L.cpu_col_reduce(n, p(M), 1, p(flags))
    assert np.flatnonzero(flags).tolist() == ref["all_isolated"]
    gid = np.unique(cl.vals[0], return_inverse=True)[1].astype(np.int32)
    L.cpu_crosscheck(n, p(M), p(gid), p(flags))
    assert np.flatnonzero(flags).tolist() == ref["user_crosscheck"]
    off = np.zeros(n + 1, np.int64)
    L.cpu_lists(n, P, p(sel), p(off), None)
    lst = np.empty(max(1, int(off[-1])), np.int32)
    L.cpu_lists(n, P, p(sel), p(off), p(lst))
    c = ctypes.c_int64()
    out = np.empty(2 * (1 << 20), np.int32)
    L.cpu_shadow(n, n, p(off), p(lst), p(alw), 1 << 20, p(out), ctypes.byref(c))
    assert c.value == ref["shadow_count"]
    assert np.array_equal(out[:2 * c.value].reshape(-1, 2), ref["shadow"].reshape(-1, 2))
