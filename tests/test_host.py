"""CPU tests of the host layer: the C ABI library loads and exports every
declared symbol, the bitarray-compatible type, interning vs the oracle's
independent interning, the YAML parser vs kano_py's parser outputs, and the
synthetic generator."""
import json
import math
import os
import re

import numpy as np
import pytest

from _golden import GOLDEN, cluster, cluster_names, expected

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# --------------------------------------------------------------------------
# C ABI
# --------------------------------------------------------------------------
def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "kano_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(kano_[a-z_0-9]+)\s*\(", hdr)))


def test_abi_library_exports_header():
    from kano import _native
    lib = _native.load()          # no GPU needed to load
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_native.SIGNATURES), set(syms) ^ set(_native.SIGNATURES)


def test_abi_no_device_is_an_error_not_a_fallback():
    from kano import _native
    if _native.gpu_available():
        pytest.skip("a GPU is visible")
    from kano._engine import DeviceBuild
    with pytest.raises(_native.KanoNativeError):
        DeviceBuild(None)


def test_model_build_fails_loudly_without_gpu():
    from kano import _native
    if _native.gpu_available():
        pytest.skip("a GPU is visible")
    from sample import paper_example
    from kano.model import ReachabilityMatrix
    cs, ps = paper_example()
    with pytest.raises(_native.KanoNativeError):
        ReachabilityMatrix.build_matrix(cs, ps)


# --------------------------------------------------------------------------
# bitarray-compatible vector
# --------------------------------------------------------------------------
def test_bitarray_subset():
    from kano._bits import BitArray
    a = BitArray("10110")
    assert len(a) == 5 and a[0] == 1 and a[1] == 0 and isinstance(a[0], int)
    assert a.count() == 3 and a.count(0) == 2
    assert a.tobytes() == b"\xb0" and a.to01() == "10110" and repr(a) == "bitarray('10110')"
    b = ~a
    assert b.to01() == "01001" and (a & b).count() == 0 and (a | b).all()
    assert (a ^ a).count() == 0 and a == BitArray("10110") and a != b
    c = BitArray(70)
    c.setall(1)
    assert c.count() == 70 and c[69] == 1
    c[69] = 0
    assert c.count() == 69 and c[-1] == 0
    assert a.tolist() == [1, 0, 1, 1, 0] and list(a) == [1, 0, 1, 1, 0]
    assert a[1:4].to01() == "011" and a.index(0) == 1 and a.search(BitArray("1")) == [0, 2, 3]
    d = a.copy()
    d &= b
    assert d.count() == 0 and a.count() == 3
    with pytest.raises(ValueError):
        a & BitArray("1")
    with pytest.raises(IndexError):
        a[5]


def test_bitarray_word_layout_roundtrip():
    from kano._bits import BitArray, bool_to_words, words_to_bool
    rng = np.random.default_rng(0)
    for n in (1, 63, 64, 65, 200):
        bits = rng.random(n) < 0.3
        w = bool_to_words(bits)
        assert w.shape[0] == (n + 63) // 64
        assert np.array_equal(words_to_bool(w, n), bits)
        s = "".join("1" if x else "0" for x in bits)
        assert BitArray(s).words().tolist() == w.tolist()


# --------------------------------------------------------------------------
# interning: product tables vs the oracle's independent interning
# --------------------------------------------------------------------------
def _eval_tables(t):
    """Evaluate sel/allow sets from product tables with numpy (test-side)."""
    n = t.n
    out = []
    for off, col, val in ((t.sel_off, t.sel_col, t.sel_val), (t.alw_off, t.alw_col, t.alw_val)):
        sets = np.ones((t.P, n), bool)
        for p in range(t.P):
            for k in range(off[p], off[p + 1]):
                sets[p] &= t.pod_val[col[k]] == val[k]
        out.append(sets)
    return out


@pytest.mark.parametrize("name", [n for n in cluster_names() if n.startswith("q_")] +
                         ["s_sparse_50", "s_broad_300"])
def test_interning_matches_reference_sets(name):
    from kano import model
    from kano._intern import intern
    from kano.synth import objects_from_json
    from _golden import rows01_to_words
    obj = cluster(name)
    exp = expected(name)
    cs, ps = objects_from_json(obj, model)
    t = intern(cs, ps)
    sel, alw = _eval_tables(t)
    n = len(cs)
    if "sel" not in exp:      # bigger records: hashes of the LSB-first words
        from _golden import sha

        def words(b):
            W = (n + 63) // 64
            buf = np.zeros((b.shape[0], W * 64), np.uint8)
            buf[:, :n] = b
            return np.packbits(buf, axis=1, bitorder="little").view("<u8")
        assert sha(words(sel)) == exp["sel_sha256"]
        assert sha(words(alw)) == exp["allow_sha256"]
        return
    want_s = np.array([[c == "1" for c in r] for r in exp["sel"]], bool).reshape(len(ps), n)
    want_a = np.array([[c == "1" for c in r] for r in exp["allow"]], bool).reshape(len(ps), n)
    assert np.array_equal(sel, want_s)
    assert np.array_equal(alw, want_a)


def test_custom_matcher_virtual_columns():
    from kano import model
    from kano._intern import intern

    class Prefix(model.LabelRelation):
        def match(self, rule, value):
            return str(value).startswith(rule)

    cs = [model.Container("a", {"app": "web-1"}), model.Container("b", {"app": "db-1"}),
          model.Container("c", {"tier": "x"})]
    p = model.Policy("p", model.PolicySelect({"app": "web"}), model.PolicyAllow({"app": "db"}),
                     model.PolicyEgress, model.PolicyProtocol([]), matcher=Prefix())
    t = intern(cs, [p])
    sel, alw = _eval_tables(t)
    assert sel[0].tolist() == [True, False, False] and alw[0].tolist() == [False, True, False]
    # the reference's own per-container predicate agrees (model.py:95-111)
    assert [p.select_policy(c) and "app" in c.labels for c in cs] == sel[0].tolist()


def test_direct_tables_equal_object_interning():
    """synth's direct integer tables describe the same sets as interning the
    materialised objects."""
    from kano import model
    from kano._intern import intern, tables_from_cluster
    from kano.synth import make_cluster, objects_from_json
    for mode in ("sparse", "broad"):
        cl = make_cluster(400, 50, mode, seed=5)
        cs, ps = objects_from_json(cl.to_json_obj(), model)
        a = _eval_tables(intern(cs, ps))
        b = _eval_tables(tables_from_cluster(cl))
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_synth_fingerprints_stable():
    from kano.synth import make_cluster
    for name in cluster_names():
        obj = cluster(name)
        if "seed" not in obj:
            continue
        s = obj["seed"]
        assert make_cluster(s["n"], s["P"], s["mode"], s["seed"]).fingerprint() == s["fingerprint"]


def test_group_ids_dict_semantics():
    from kano import model
    from kano._intern import group_ids
    cs = [model.Container(str(i), l) for i, l in enumerate(
        [{"u": 1}, {"u": True}, {"u": 1.0}, {}, {"u": ""}, {"u": "x"}])]
    assert group_ids(cs, "u").tolist() == [0, 0, 0, 1, 1, 2]


def _py_intern(cs, ps, monkeypatch):
    """intern() with the native passes switched off (the per-pod Python loops)."""
    from kano import _intern as I

    class Off:
        def __getattr__(self, name):
            def f(*a):
                raise TypeError("native pass off")
            return f
    with monkeypatch.context() as m:
        m.setattr(I, "_kano_host", Off())
        return I.intern(cs, ps)


def _same_tables(a, b):
    assert a.n == b.n and a.ncols == b.ncols
    for f in ("pod_val", "sel_off", "sel_col", "sel_val", "alw_off", "alw_col", "alw_val"):
        x, y = getattr(a, f), getattr(b, f)
        assert x.dtype == y.dtype and np.array_equal(x, y), f
    assert list(a.state.keys) == list(b.state.keys)
    assert a.state.col_of_key == b.state.col_of_key
    for c, idx in a.state.indexes.items():
        assert idx.ids == b.state.indexes[c].ids and idx.next_id == b.state.indexes[c].next_id


@pytest.mark.parametrize("seed", range(6))
def test_native_interning_equals_python_loops(seed, monkeypatch):
    """csrc/kano_hostext.c (scan_labels, policy_terms, intern_column) against
    intern's own per-pod / per-term loops on awkward values: NaN (float and
    numpy, shared and distinct objects), 1 / 1.0 / True collapsing, None, a
    key no pod carries (quirk Q1), rules no pod value equals, unhashable rule
    values, and -- for seeds >= 3 -- an unhashable pod value and a custom
    matcher, which send the columns / terms to the loops."""
    from kano import model
    from kano._intern import intern
    rng = np.random.default_rng(seed)
    nan = float("nan")
    pool = [1, 1.0, True, 0, False, "a", "b", None, nan, float("nan"), np.float64("nan"), 2.5, "1"]
    if seed >= 3:
        pool.append(["unhashable"])
    keys = ["k0", "k1", "k2", "k3"]
    cs = []
    for i in range(300):
        lab = {k: pool[rng.integers(len(pool))] for k in keys if rng.random() < 0.7}
        cs.append(model.Container(f"c{i}", lab))
    rules = [1, True, "a", "zz", nan, None, ["x"], 2.5]
    ps = []
    for p in range(60):
        sel = {k: rules[rng.integers(len(rules))] for k in keys + ["absent"] if rng.random() < 0.4}
        alw = {k: rules[rng.integers(len(rules))] for k in keys if rng.random() < 0.4}
        kw = {}
        if seed >= 3 and p % 17 == 5:
            class Loose(model.DefaultEqualityLabelRelation):
                def match(self, rule, value):
                    return str(rule) == str(value)
            kw["matcher"] = Loose()
        ps.append(model.Policy(f"p{p}", model.PolicySelect(sel), model.PolicyAllow(alw),
                               model.PolicyIngress if p % 3 == 0 else model.PolicyEgress,
                               model.PolicyProtocol(["TCP"]), **kw))
    _same_tables(intern(cs, ps), _py_intern(cs, ps, monkeypatch))


def test_native_group_ids_equal_loop(monkeypatch):
    from kano import model, _intern as I
    rng = np.random.default_rng(3)
    pool = [1, 1.0, True, "", "x", None, 2.5]
    cs = [model.Container(str(i), {"u": pool[rng.integers(len(pool))]} if rng.random() < 0.8
                          else {}) for i in range(500)]
    got = I.group_ids(cs, "u")
    with monkeypatch.context() as m:
        m.setattr(I._kano_host, "group_ids", lambda *a: (_ for _ in ()).throw(ValueError()))
        assert np.array_equal(got, I.group_ids(cs, "u"))


# --------------------------------------------------------------------------
# parser vs kano_py's parser (tests/golden/expected/parser.json)
# --------------------------------------------------------------------------
def test_parser_matches_reference(capsys):
    from kano.parser import ConfigParser
    recs = json.load(open(os.path.join(GOLDEN, "expected", "parser.json")))
    ydir = os.path.join(GOLDEN, "yaml")
    for rec in recs:
        cp = ConfigParser()
        cp.parse(os.path.join(ydir, rec["file"]))
        out = capsys.readouterr().out.replace(ydir, "<YAML>")
        assert out == rec["stdout"], rec["file"]
        assert [repr(c.labels) for c in cp.containers] == rec["containers_repr"]
        assert [c.name for c in cp.containers] == [c[0] for c in rec["containers"]]
        got = [[q.name, None if q.selector.labels is None else repr(q.selector.labels),
                None if q.allow.labels is None else repr(q.allow.labels),
                q.direction.direction, q.protocol] for q in cp.policies]
        assert got == rec["policies"], rec["file"]


def test_parser_shares_labels_and_walks_directory(tmp_path, capsys):
    from kano.parser import ConfigParser
    src = os.path.join(GOLDEN, "yaml")
    for f in ("pod_two_containers.yaml", "np_egress_ports.yaml"):
        (tmp_path / f).write_text(open(os.path.join(src, f)).read())
    cp = ConfigParser(str(tmp_path))
    cs, ps = cp.parse()
    assert len(cs) == 2 and cs[0].labels is cs[1].labels          # quirk Q9
    assert [p.name for p in ps] == ["web-out-ingress", "web-out-egress"]
    assert ps[1].protocol == ["TCP", 5432]
    assert ConfigParser().parse() is None
    assert "no filepath specified" in capsys.readouterr().out


# --------------------------------------------------------------------------
# wave_transpose64 (csrc/kano_kernels.hpp): the butterfly, lane by lane
# --------------------------------------------------------------------------
def _wave_transpose64_model(x):
    """The kernel's six stages on 64 lanes' words: stage s pairs lanes r and
    r ^ s; the lower lane keeps its bits c with c & s == 0 and takes the
    partner's into c | s, the upper lane the converse (kano_kernels.hpp,
    wave_transpose64)."""
    masks = [0x00000000ffffffff, 0x0000ffff0000ffff, 0x00ff00ff00ff00ff,
             0x0f0f0f0f0f0f0f0f, 0x3333333333333333, 0x5555555555555555]
    full = (1 << 64) - 1
    x = [int(v) for v in x]
    for k, m in enumerate(masks):
        s = 32 >> k
        y = [x[r ^ s] for r in range(64)]
        x = [((x[r] & ~m & full) | ((y[r] & ~m & full) >> s)) if r & s
             else ((x[r] & m) | (((y[r] & m) << s) & full)) for r in range(64)]
    return x


def test_wave_transpose64_butterfly_is_the_transpose():
    rng = np.random.default_rng(7)
    for density in (0.5, 0.05, 0.95):
        bits = rng.random((64, 64)) < density
        rows = [sum(1 << c for c in range(64) if bits[r, c]) for r in range(64)]
        out = _wave_transpose64_model(rows)
        for r in range(64):
            assert out[r] == sum(1 << j for j in range(64) if bits[j, r]), (density, r)
