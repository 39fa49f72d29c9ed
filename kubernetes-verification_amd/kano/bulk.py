"""Bulk YAML front end: a directory of pod and
NetworkPolicy files straight to the engine's integer tables, parsed and
interned in a process pool.

``ConfigParser.parse`` (kano_py/kano/parser.py:17-82, restated in
kano/parser.py) loads one document per file with PyYAML and builds Python
objects one file at a time; ``intern`` (kano/_intern.py) then walks every
container's labels.  At 1M pods both are single-core Python.  Here workers
take contiguous runs of the walk's files, convert them exactly as
``create_object`` does (one Policy per ingress / egress rule, allow = the
podSelector of the rule's LAST peer that has one, one Container per
``spec.containers`` entry sharing the pod's labels: quirks Q8, Q9) and intern
the container labels locally (value -> id under Python ==, NaN never
matches).  The parent concatenates in walk order and merges the per-worker
value tables, so the result equals ``intern(*ConfigParser().parse(path))``
array for array, column order and value ids included
(tests/test_bulk.py).

Errors follow the reference: a file that fails to load or convert in file
mode prints "Error opening or reading file <path>" and keeps what it
appended; in directory mode the first bad file (in walk order) ends the walk
with "Error opening or reading directory", keeping everything before it,
including what the bad file appended before failing.  A policy without an
allow side (a namespaceSelector-only rule) raises the AttributeError that
``build_matrix`` raises on it (model.py:145), here at load time.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from yaml import load

try:
    from yaml import CLoader as Loader
except ImportError:  # pragma: no cover
    from yaml import Loader

from ._intern import ABSENT, NEVER_MATCH_VALUE, Tables, _ValueIndex


@dataclass
class BulkCluster:
    tables: Tables
    container_names: List[Any]
    policy_names: List[Any]
    groups: Optional[np.ndarray]     # user_hashmap ids of `label` (None without label)
    files: int


# ---------------------------------------------------------------------------
# walk order and per-file conversion (kano_py/kano/parser.py:23-82)
# ---------------------------------------------------------------------------
def walk_files(path: str) -> List[str]:
    if os.path.isfile(path):
        return [path]
    out = []
    for subdir, _dirs, files in os.walk(path):
        for name in files:
            out.append(os.path.join(subdir, name))
    return out


def _rule_allow(peers):
    allow, ports = None, None
    for peer in peers:
        if "podSelector" in peer:
            allow = peer["podSelector"]["matchLabels"]
        if "ports" in peer:
            ports = [peer["ports"]["protocol"], peer["ports"]["port"]]
    return allow, ports


def _convert(data, pods: list, pols: list) -> None:
    """create_object (parser.py:51-82), appending records as it goes so that
    a failure part-way keeps what the reference would have kept."""
    kind = data["kind"]
    if kind == "NetworkPolicy":
        spec = data["spec"]
        select = spec["podSelector"]["matchLabels"]
        name = data["metadata"]["name"]
        for ptype, rules_key, peers_key, suffix, ingress in (
                ("Ingress", "ingress", "from", "-ingress", True),
                ("Egress", "egress", "to", "-egress", False)):
            if ptype not in spec["policyTypes"]:
                continue
            for rule in spec[rules_key]:
                allow, _ports = _rule_allow(rule[peers_key])
                pols.append((name + suffix, select, allow, ingress))
    elif kind == "Pod":
        labels = data["metadata"]["labels"]
        for c in data["spec"]["containers"]:
            pods.append((c["name"], labels))


class _LocalValues:
    """One worker's value table of a key: ids in first-appearance order."""

    __slots__ = ("index", "uniques", "pos", "ids")

    def __init__(self):
        self.index = _ValueIndex()
        self.uniques: List[Any] = []
        self.pos: List[int] = []
        self.ids: List[int] = []

    def add(self, i: int, v) -> None:
        vid = self.index.pod_id(v)
        if vid >= 0 and vid == len(self.uniques):
            self.uniques.append(v)
        self.pos.append(i)
        self.ids.append(vid)


def _parse_chunk(args):
    files, single, label = args
    pods: list = []
    pols: list = []
    error = None
    for fi, path in enumerate(files):
        try:
            with open(path) as f:
                data = load(f, Loader=Loader)
            _convert(data, pods, pols)
        except Exception:  # noqa: BLE001  (the reference's bare except)
            error = fi
            if not single:
                break
    # local interning of the container labels
    keys: Dict[Any, _LocalValues] = {}
    for i, (_name, labels) in enumerate(pods):
        for k, v in labels.items():
            lv = keys.get(k)
            if lv is None:
                lv = keys[k] = _LocalValues()
            lv.add(i, v)
    key_data = [(k, lv.uniques, np.asarray(lv.pos, np.int32), np.asarray(lv.ids, np.int32))
                for k, lv in keys.items()]
    # user_hashmap groups of `label` (algorithm.py:20-24): value or "", dict
    # semantics; values unequal to themselves (NaN objects) are their own group
    groups = None
    if label is not None:
        gmap: Dict[Any, int] = {}
        guniq: List[Any] = []
        gids = np.empty(len(pods), np.int32)
        for i, (_name, labels) in enumerate(pods):
            v = labels.get(label, "")
            try:
                private = v != v
            except Exception:  # noqa: BLE001
                private = False
            if private:
                gids[i] = len(guniq)
                guniq.append(("private", v))
                continue
            g = gmap.get(v)      # unhashable values raise TypeError, as in the reference
            if g is None:
                g = gmap[v] = len(guniq)
                guniq.append(("value", v))
            gids[i] = g
        groups = (guniq, gids)
    names = [name for name, _ in pods]
    return dict(n=len(pods), names=names, keys=key_data, pols=pols, error=error, groups=groups)


# ---------------------------------------------------------------------------
# parent: concatenate in walk order, merge value tables, emit Tables
# ---------------------------------------------------------------------------
def _hip_loaded() -> bool:
    try:
        with open("/proc/self/maps") as f:
            return "libamdhip64" in f.read()
    except OSError:
        return True


def _split(files: Sequence[str], parts: int) -> List[List[str]]:
    parts = max(1, min(parts, len(files)))
    step = (len(files) + parts - 1) // parts
    return [list(files[i:i + step]) for i in range(0, len(files), step)]


def load_tables(path: str, workers: Optional[int] = None, label=None,
                chunks_per_worker: int = 4) -> BulkCluster:
    """ConfigParser(path).parse() + intern(), in a process pool of `workers`
    (default: the usable cores, at most 16; 1 = in this process)."""
    if path is None:
        print("no filepath specified")
        raise ValueError("no filepath specified")
    single = os.path.isfile(path)
    files = walk_files(path)
    if workers is None:
        workers = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                             else (os.cpu_count() or 1)))
    chunks = _split(files, workers * chunks_per_worker) if files else []
    jobs = [(c, single, label) for c in chunks]
    if workers > 1 and len(jobs) > 1:
        import multiprocessing as mp
        # fork is cheapest; a process that already holds a GPU runtime starts
        # clean workers instead (they only parse YAML)
        ctx = mp.get_context("spawn" if _hip_loaded() else "fork")
        with ctx.Pool(workers) as pool:
            parts = pool.map(_parse_chunk, jobs, chunksize=1)
    else:
        parts = [_parse_chunk(j) for j in jobs]

    # the walk stops at the first bad file (directory mode); file mode keeps
    # the partial result of its one file
    kept = []
    for ci, part in enumerate(parts):
        kept.append(part)
        if part["error"] is not None:
            if single:
                print("Error opening or reading file " + path)
            else:
                print("Error opening or reading directory")
            break

    offs = np.cumsum([0] + [p["n"] for p in kept])
    n = int(offs[-1])
    names: List[Any] = [nm for p in kept for nm in p["names"]]
    pols = [q for p in kept for q in p["pols"]]

    # KEYS: every label key of a container, first appearance in walk order
    KEYS: Dict[Any, None] = {}
    for p in kept:
        for k, _u, _pos, _ids in p["keys"]:
            KEYS.setdefault(k, None)

    # working sides (model.py:82-93): ingress swaps select and allow
    col_of_key: Dict[Any, int] = {}
    col_keys: List[Any] = []

    def key_col(k) -> int:
        c = col_of_key.get(k)
        if c is None:
            c = col_of_key[k] = len(col_keys)
            col_keys.append(k)
        return c

    raw_terms = []
    for _name, select, allow, ingress in pols:
        ws, wa = (allow, select) if ingress else (select, allow)
        per_side = []
        for side in (ws, wa):
            terms = []
            for k, rule in side.items():     # None side: AttributeError as build_matrix
                if k not in KEYS:
                    continue                  # quirk Q1
                terms.append((key_col(k), rule))
            per_side.append(terms)
        raw_terms.append(per_side)

    ncols = len(col_keys)
    pod_val = np.full((ncols, n), ABSENT, dtype=np.int32)
    indexes = [_ValueIndex() for _ in range(ncols)]
    for w, p in enumerate(kept):
        base = int(offs[w])
        for k, uniques, pos, ids in p["keys"]:
            c = col_of_key.get(k)
            if c is None:
                continue
            remap = np.asarray([indexes[c].pod_id(v) for v in uniques] + [NEVER_MATCH_VALUE],
                               dtype=np.int32)
            local = np.where(ids >= 0, ids, len(uniques))
            pod_val[c, base + pos] = remap[local]

    def csr(which: int):
        off = np.zeros(len(raw_terms) + 1, dtype=np.int64)
        cols: List[int] = []
        vals: List[int] = []
        for pi, per_side in enumerate(raw_terms):
            for col, rule in per_side[which]:
                cols.append(col)
                vals.append(indexes[col].rule_id(rule))
            off[pi + 1] = len(cols)
        return off, np.asarray(cols, dtype=np.int32), np.asarray(vals, dtype=np.int32)

    so, sc, sv = csr(0)
    ao, ac, av = csr(1)
    tables = Tables(n, ncols, pod_val, so, sc, sv, ao, ac, av)

    groups = None
    if label is not None:
        gmap: Dict[Any, int] = {}
        gcount = 0
        gids = np.empty(n, np.int32)
        for w, p in enumerate(kept):
            guniq, local = p["groups"]
            remap = np.empty(len(guniq), np.int32)
            for u, (kind, v) in enumerate(guniq):
                if kind == "private":
                    remap[u] = gcount
                    gcount += 1
                    continue
                g = gmap.get(v)
                if g is None:
                    g = gmap[v] = gcount
                    gcount += 1
                remap[u] = g
            gids[int(offs[w]):int(offs[w + 1])] = remap[local]
        groups = gids
    return BulkCluster(tables, names, [q[0] for q in pols], groups, len(files))


def write_cluster_yaml(cl, directory: str) -> int:
    """Write a synth.Cluster as kano YAML, one Pod or NetworkPolicy document
    per file as the reference's generator writes them
    (kano_py/tests/generate.py:53-86): pod<i> with one container c<i>; pol<p>
    with the podSelector and one ingress / egress rule whose single peer
    podSelector is the allow side.  Label values are the generator's strings
    ("ns3", "app12", ...), plain YAML scalars.  Returns the file count."""
    os.makedirs(directory, exist_ok=True)

    def mapping(d: dict, indent: str) -> str:
        if not d:
            return " {}\n"
        return "\n" + "".join(f"{indent}{k}: {v}\n" for k, v in d.items())

    nfiles = 0
    for i in range(cl.n):
        doc = ("apiVersion: v1\nkind: Pod\nmetadata:\n  name: pod%d\n  labels:%s"
               "spec:\n  containers:\n  - name: c%d\n    image: busybox\n"
               % (i, mapping(cl.pod_labels(i), "    "), i))
        with open(os.path.join(directory, f"pod{i:07d}.yml"), "w") as f:
            f.write(doc)
        nfiles += 1
    for p in range(cl.P):
        sel = cl._side(cl.pols_off, cl.pols_key, cl.pols_val, p)
        alw = cl._side(cl.pola_off, cl.pola_key, cl.pola_val, p)
        ptype, rules, peers = (("Ingress", "ingress", "from") if cl.ingress[p]
                               else ("Egress", "egress", "to"))
        doc = ("apiVersion: networking.k8s.io/v1\nkind: NetworkPolicy\nmetadata:\n"
               "  name: pol%d\n  namespace: default\nspec:\n  podSelector:\n    matchLabels:%s"
               "  policyTypes:\n  - %s\n  %s:\n  - %s:\n    - podSelector:\n        matchLabels:%s"
               % (p, mapping(sel, "      "), ptype, rules, peers, mapping(alw, "          ")))
        with open(os.path.join(directory, f"pol{p:07d}.yml"), "w") as f:
            f.write(doc)
        nfiles += 1
    return nfiles


__all__ = ["BulkCluster", "load_tables", "walk_files", "write_cluster_yaml"]
