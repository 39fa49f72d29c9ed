"""The bulk YAML front end (kano/bulk.py) against the
drop-in parser + interning it replaces: ConfigParser.parse (whose output is
pinned to kano_py's own parser by tests/golden/expected/parser.json,
test_host.py) followed by intern().  Equal arrays, equal names, equal error
behaviour, for one worker and for a process pool."""
import os
import shutil

import numpy as np
import pytest

from conftest import GOLDEN

FIELDS = ("pod_val", "sel_off", "sel_col", "sel_val", "alw_off", "alw_col", "alw_val")


def reference(path, label=None):
    from kano.parser import ConfigParser
    from kano._intern import intern, group_ids
    cs, ps = ConfigParser(path).parse()
    t = intern(cs, ps)
    g = group_ids(cs, label) if label is not None else None
    return cs, ps, t, g


def assert_same(b, cs, ps, t, g):
    assert b.tables.n == t.n and b.tables.ncols == t.ncols
    for f in FIELDS:
        assert np.array_equal(getattr(b.tables, f), getattr(t, f)), f
    assert b.container_names == [c.name for c in cs]
    assert b.policy_names == [p.name for p in ps]
    if g is not None:
        assert np.array_equal(b.groups, g)


@pytest.mark.parametrize("workers", [1, 3])
@pytest.mark.parametrize("mode,seed", [("sparse", 21), ("broad", 22)])
def test_generated_directory(tmp_path, mode, seed, workers):
    from kano import bulk
    from kano.synth import make_cluster
    cl = make_cluster(600, 90, mode, seed=seed)
    d = str(tmp_path / "y")
    assert bulk.write_cluster_yaml(cl, d) == cl.n + cl.P
    b = bulk.load_tables(d, workers=workers, label="tenant")
    assert_same(b, *reference(d, "tenant"))


MIXED = {
    "p1.yml": "kind: Pod\nmetadata:\n  labels: {a: on, b: 1, c: 1.0, d: .nan, e: [1, 2]}\n"
              "spec:\n  containers:\n  - name: x1\n  - name: x2\n",
    "p2.yml": "kind: Pod\nmetadata:\n  labels: {a: true, b: '1', c: 1, d: .nan, e: [1, 2]}\n"
              "spec:\n  containers:\n  - name: y1\n",
    "p3.yml": "kind: Pod\nmetadata:\n  labels: {a: off, b: 2, f: yes}\n"
              "spec:\n  containers:\n  - name: z1\n",
    "q1.yml": "kind: NetworkPolicy\nmetadata: {name: n1}\nspec:\n  podSelector:\n"
              "    matchLabels: {a: 1, zz: q}\n  policyTypes: [Ingress, Egress]\n"
              "  ingress:\n  - from:\n    - podSelector: {matchLabels: {b: 1}}\n"
              "    - podSelector: {matchLabels: {c: 1}}\n"
              "  egress:\n  - to:\n    - podSelector: {matchLabels: {e: [1, 2]}}\n",
    "q2.yml": "kind: NetworkPolicy\nmetadata: {name: n2}\nspec:\n  podSelector:\n"
              "    matchLabels: {d: .nan}\n  policyTypes: [Egress]\n"
              "  egress:\n  - to:\n    - podSelector: {matchLabels: {f: true}}\n",
}


@pytest.mark.parametrize("workers", [1, 2, 5])
def test_yaml_typing_and_quirks(tmp_path, workers):
    """YAML 1.1 typing (on/yes -> True, 1 vs '1' vs 1.0), NaN never matching,
    list values, last podSelector peer wins, unknown selector keys dropped,
    containers sharing their pod's labels."""
    from kano import bulk
    d = tmp_path / "m"
    d.mkdir()
    for name, text in MIXED.items():
        (d / name).write_text(text)
    b = bulk.load_tables(str(d), workers=workers, label="a")
    assert_same(b, *reference(str(d), "a"))


def test_bad_file_stops_the_walk(tmp_path, capsys):
    """Directory mode: the first bad file in walk order ends the walk,
    keeping everything before it (kano_py/kano/parser.py:40-47)."""
    from kano import bulk
    from kano.synth import make_cluster
    cl = make_cluster(200, 30, "sparse", seed=23)
    d = str(tmp_path / "y")
    bulk.write_cluster_yaml(cl, d)
    files = bulk.walk_files(d)
    bad = files[len(files) // 2]
    shutil.copy(os.path.join(GOLDEN, "yaml", "broken.yaml"), bad)
    ref = reference(d)
    ref_out = capsys.readouterr().out
    for workers in (1, 4):
        b = bulk.load_tables(d, workers=workers)
        assert capsys.readouterr().out == ref_out
        assert_same(b, *ref)


def test_golden_yaml_files(capsys):
    """Every fixture of tests/golden/yaml in file mode, including the broken
    one and the namespaceSelector-only rule whose allow side is None (the
    AttributeError that build_matrix raises, model.py:145)."""
    from kano import bulk
    from kano.parser import ConfigParser
    from kano._intern import intern
    ydir = os.path.join(GOLDEN, "yaml")
    for name in sorted(os.listdir(ydir)):
        path = os.path.join(ydir, name)
        cs, ps = ConfigParser(path).parse()
        ref_out = capsys.readouterr().out
        try:
            t = intern(cs, ps)
        except AttributeError as e:
            with pytest.raises(AttributeError, match=str(e).replace("'", ".")):
                bulk.load_tables(path, workers=1)
            capsys.readouterr()
            continue
        b = bulk.load_tables(path, workers=1)
        assert capsys.readouterr().out == ref_out, name
        assert_same(b, cs, ps, t, None)


@pytest.mark.gpu
def test_bulk_tables_build_the_same_matrix(tmp_path):
    """YAML directory -> bulk tables -> GPU verify equals the drop-in object
    path (ConfigParser -> Container / Policy -> build_matrix) and the oracle."""
    from kano import bulk
    from kano._engine import DeviceBuild
    from kano.synth import make_cluster
    from oracle import kano_oracle as orc
    cl = make_cluster(1500, 200, "sparse", seed=24)
    d = str(tmp_path / "y")
    bulk.write_cluster_yaml(cl, d)
    b = bulk.load_tables(d, workers=2, label="tenant")   # spawned workers: HIP is loaded
    cs, ps, t, g = reference(d, "tenant")
    e1 = DeviceBuild(b.tables)
    e2 = DeviceBuild(t)
    n = t.n
    assert np.array_equal(e1.rows(0, n), e2.rows(0, n))
    # the oracle on the same objects, in the walk's order (os.walk lists a
    # directory in no fixed order, so pod i is not pod<i>)
    obj = {"pods": [{"name": c.name, "labels": c.labels} for c in cs],
           "policies": [{"name": q.name, "select": q.selector.labels, "allow": q.allow.labels,
                         "direction": "ingress" if q.direction.is_ingress() else "egress"}
                        for q in ps]}
    ref = orc.run_c(obj, label="tenant")
    assert np.array_equal(e1.rows(0, n), ref["M"])
    r = e1.verify(b.groups, sys_row=0, shadow=True)
    assert r["user_crosscheck"].tolist() == ref["user_crosscheck"]
    assert np.array_equal(np.ascontiguousarray(r["pairs"]).reshape(-1, 2), ref["shadow"])
    e1.close()
    e2.close()
