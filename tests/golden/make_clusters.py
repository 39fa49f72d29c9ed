"""Write the input clusters of the golden vectors (run with the repo's python3).

    python3 tests/golden/make_clusters.py

Produces tests/golden/clusters/*.json: hand-written quirk clusters (SURVEY.md
§A.4) and small seeded clusters from kano/synth.py.  The larger seeded
clusters (C2: 10k pods / 1k policies) are regenerated from their seed by the
tests; their fingerprint is stored next to the expected outputs.
tests/golden/make_golden.py then runs kano_py itself on these inputs.
"""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "kubernetes-verification_amd"))

from kano.synth import make_cluster  # noqa: E402

OUT = os.path.join(HERE, "clusters")


def pol(name, select, allow, direction="ingress"):
    return {"name": name, "select": select, "allow": allow, "direction": direction,
            "protocol": ["TCP", "80"]}


def pod(name, **labels):
    return {"name": name, "labels": labels}


QUIRKS = {
    # Q1: selector/allow keys carried by no pod are ignored (match all)
    "q_unknown_key": {
        "label": "app",
        "pods": [pod("a", app="x"), pod("b", app="y"), pod("c", app="x", tier="db")],
        "policies": [pol("p0", {"zz": "q"}, {"app": "x"}, "egress"),
                     pol("p1", {"app": "y", "zz": "q"}, {"zz": "r"}, "egress"),
                     pol("p2", {"tier": "db"}, {"nope": 1, "app": "y"}, "ingress")],
    },
    # Q7: Python == across int / float / bool / str / None values
    "q_types": {
        "label": "v",
        "pods": [pod("i1", v=1), pod("f1", v=1.0), pod("b1", v=True), pod("s1", v="1"),
                 pod("n0", v=None), pod("i0", v=0), pod("bf", v=False), pod("f25", v=2.5)],
        "policies": [pol("p_int", {"v": 1}, {"v": 0}, "egress"),
                     pol("p_str", {"v": "1"}, {"v": None}, "egress"),
                     pol("p_true", {"v": True}, {"v": 2.5}, "ingress"),
                     pol("p_none", {"v": None}, {"v": False}, "ingress"),
                     pol("p_zero", {"v": 0.0}, {"v": "1"}, "egress")],
    },
    # Q2: ingress/egress side swap, empty selector dicts match everything
    "q_dirs": {
        "label": "team",
        "pods": [pod("w", role="web", team="a"), pod("d", role="db", team="a"),
                 pod("c", role="cache", team="b"), pod("x", team="b"), pod("y", role="web")],
        "policies": [pol("e1", {"role": "web"}, {"role": "db"}, "egress"),
                     pol("i1", {"role": "web"}, {"role": "db"}, "ingress"),
                     pol("all", {}, {"team": "b"}, "egress"),
                     pol("none", {"role": "nope"}, {}, "ingress"),
                     pol("i2", {}, {}, "ingress")],
    },
    # Q4: equal allow sets shadow each other both ways; an empty allow set is a
    # subset of every set; duplicates per container
    "q_shadow": {
        "label": "g",
        "pods": [pod("p%d" % i, app="a" if i < 4 else "b", g=str(i % 3), k=i % 2) for i in range(8)],
        "policies": [pol("s1", {"app": "a"}, {"k": 0}, "egress"),
                     pol("s2", {"app": "a"}, {"k": 0}, "egress"),
                     pol("s3", {"app": "a"}, {"k": 5}, "egress"),
                     pol("s4", {"k": 1}, {"app": "b"}, "egress"),
                     pol("s5", {"k": 1}, {"app": "b", "k": 1}, "egress"),
                     pol("s6", {"app": "b"}, {}, "egress")],
    },
    # Q6: a missing crosscheck label groups with the literal "" value
    "q_missing_label": {
        "label": "user",
        "pods": [pod("a", user="u1", r="x"), pod("b", r="x"), pod("c", user="", r="y"),
                 pod("d", user="u2", r="y"), pod("e", r="z")],
        "policies": [pol("x_to_y", {"r": "x"}, {"r": "y"}, "egress"),
                     pol("y_to_z", {"r": "y"}, {"r": "z"}, "egress"),
                     pol("z_to_x", {"r": "z"}, {"r": "x"}, "ingress")],
    },
    # one light row class selected by more policies than k_rows' LDS segment
    # table holds (ROWS_SEG = 256): 320 policies select the "hot" pods, each
    # allowing one pod (duplicates every 300 -> shadow pairs), so the class
    # stays light (its rebuild scatters 320 entries) and takes the
    # non-segmented walk over the flat lists
    "q_wide_select": {
        "label": "grp",
        "pods": [pod("p%d" % i, id="p%d" % i, grp="hot" if i % 120 == 7 else "g%d" % (i % 5),
                     app="a%d" % (i % 9)) for i in range(1200)],
        "policies": ([pol("w%d" % k, {"grp": "hot"}, {"id": "p%d" % (k % 300)}, "egress")
                      for k in range(320)] +
                     [pol("x%d" % k, {"app": "a%d" % (k % 9)}, {"grp": "g%d" % (k % 5)},
                          "ingress" if k % 2 else "egress") for k in range(20)]),
    },
    # every container selected by at most one policy: policy_conflict returns []
    "q_no_conflict": {
        "label": "app",
        "pods": [pod("a", app="1"), pod("b", app="2"), pod("c", app="3")],
        "policies": [pol("p", {"app": "1"}, {"app": "2"}, "egress"),
                     pol("q", {"app": "2"}, {"app": "3"}, "egress")],
    },
    # NaN never equals anything; list values compare with ==
    "q_nan_list": {
        "label": "app",
        "pods": [pod("a", app="x", v=float("nan"), l=[1, 2]), pod("b", app="x", v=1.5, l=[1, 2]),
                 pod("c", app="y", v=float("nan"), l=[3])],
        "policies": [pol("nan_rule", {"v": float("nan")}, {"app": "x"}, "egress"),
                     pol("list_rule", {"l": [1, 2]}, {"app": "y"}, "egress"),
                     pol("num_rule", {"v": 1.5}, {"l": [3]}, "ingress")],
    },
}

SEEDED = [  # name, n, P, mode, seed, label
    ("s_sparse_50", 50, 10, "sparse", 100, "tenant"),
    ("s_sparse_200", 200, 40, "sparse", 101, "tenant"),
    ("s_broad_300", 300, 30, "broad", 102, "tenant"),
    ("s_sparse_500", 500, 50, "sparse", 103, "ns"),
    ("s_sparse_1000", 1000, 100, "sparse", 104, "tenant"),
    ("s_broad_1000", 1000, 60, "broad", 105, "tenant"),
    ("s_sparse_2000", 2000, 200, "sparse", 106, "app"),
]


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, obj in QUIRKS.items():
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump(obj, f, indent=1)
    for name, n, P, mode, seed, label in SEEDED:
        cl = make_cluster(n, P, mode, seed)
        obj = cl.to_json_obj()
        obj["label"] = label
        obj["seed"] = dict(n=n, P=P, mode=mode, seed=seed, fingerprint=cl.fingerprint())
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump(obj, f, separators=(",", ":"))
    print("wrote", len(QUIRKS) + len(SEEDED), "clusters to", OUT)
    if "--big" in sys.argv:
        # C2/C3/C4 (BASELINE.json configs[1..3]): regenerated from their seeds
        # by the tests; only kano_py's outputs on them are committed
        from kano.synth import make_config
        names = [a for a in sys.argv[1:] if not a.startswith("--")] or ["C2"]
        for name in names:
            cl = make_config(name)
            obj = cl.to_json_obj()
            obj["label"] = "tenant"
            obj["seed"] = dict(n=cl.n, P=cl.P, mode=cl.mode, seed=cl.seed,
                               fingerprint=cl.fingerprint())
            with open(f"/tmp/kano_golden_{name}.json", "w") as f:
                json.dump(obj, f, separators=(",", ":"))
            print(f"wrote /tmp/kano_golden_{name}.json")


if __name__ == "__main__":
    assert math.isnan(float("nan"))
    main()
