"""Seeded synthetic cluster generator (numpy PCG64) for the Kano benchmark configs.

The reference ships only an unseeded, uniform generator
(`kano_py/tests/generate.py:5-96`: random pods with a `User` label plus 0-4
`keyX: valueY` labels; each policy copies the labels of two random pods into
its podSelector / peer podSelector).  That generator saturates (matrix
density 1.0 at 20k pods), so the benchmark configs C2-C5
(BASELINE.json) use this generator instead.  It keeps the reference's policy
construction -- a policy's two label dicts are copied from two random pods --
and draws the pod labels from Zipf-like popularity laws:

* ``ns``     namespaces, Zipf s=1.1 over max(16, n/1000) values;
* ``app``    deployments, Zipf-Mandelbrot s=1.3, q=50 over n/20 values.  Every
             app lives in one namespace (its pods inherit ``ns``), so the
             podSelector ``{ns, app}`` names one deployment.  The Mandelbrot
             offset keeps the largest app near 1% of the pods; with the plain
             Zipf law the survey sketched, the top app holds 27% of all pods
             and policy_shadow's output exceeds 10^9 tuples at 100k pods;
* ``tenant`` Zipf s=1.2 over 64 values, drawn per namespace;
* ``role``   uniform over 8 values, drawn per pod;
* 0-3 extra ``kX: vY`` labels (32 keys, 16 values each, Zipf s=1.1).

Policies pick ingress/egress with p=0.5.  ``sparse`` (C2, C3, C5): select =
{ns, app} of pod a (+ role w.p. 0.5), allow = {ns, app} of pod b.  ``broad``
(C4): select = {ns} of a, allow = {ns} or {tenant} of b.  Each policy side
gets, w.p. 1%, an extra term whose key no pod carries (exercises quirk Q1,
`kano_py/kano/model.py:143,146`).

``dense`` (D1, the MFMA crossover sweep): egress only, ``tenants`` uniform
tenants and ``apps`` uniform apps drawn independently per pod; a share
``broad`` of the policies select and allow {tenant} of a (intra-tenant), the
rest select {tenant, app} of a and allow {tenant, app} of b (which makes
(tenant, app) the row and column classes).  Every row class is then selected by ~broad*P/tenants
policies: the class x policy selector matrix is dense, the regime where the
int8 MFMA contraction beats the bitwise OR ("The dense path").

The generator emits integer tables directly (what the engine consumes) and can
materialise the same cluster as kano API objects / JSON, so the host interning
path and the direct-table path are checked against each other in tests.
"""
from __future__ import annotations

import hashlib
import json
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

N_EXTRA_KEYS = 32
N_EXTRA_VALS = 16
N_TENANTS = 64
N_ROLES = 8
FIXED_KEYS = ["tenant", "ns", "app", "role"]
KEY_NAMES = FIXED_KEYS + [f"k{i}" for i in range(N_EXTRA_KEYS)]
VALUE_PREFIX = {"tenant": "t", "ns": "ns", "app": "app", "role": "r"}
ABSENT_KEY = "zz-absent"          # a key no pod carries (quirk Q1)
ABSENT_VAL = "x"

K_TENANT, K_NS, K_APP, K_ROLE = 0, 1, 2, 3

CONFIGS = {
    # name: (pods, policies, mode, seed) -- BASELINE.json configs[1..4]
    "C2": (10_000, 1_000, "sparse", 0),
    "C3": (100_000, 10_000, "sparse", 1),
    "C4": (100_000, 10_000, "broad", 2),
    "C5": (1_000_000, 100_000, "sparse", 3),
    # the dense-path config (not in BASELINE.json: the MFMA crossover's bench line)
    "D1": (100_000, 10_000, "dense", 4, {"tenants": 4, "apps": 2000, "broad": 0.9}),
}


def _zipf_weights(m: int, s: float, q: float = 0.0) -> np.ndarray:
    r = np.arange(1, m + 1, dtype=np.float64)
    w = (r + q) ** (-s)
    return w / w.sum()


def value_name(key_idx: int, vid: int) -> str:
    if key_idx < len(FIXED_KEYS):
        return f"{VALUE_PREFIX[FIXED_KEYS[key_idx]]}{vid}"
    return f"v{vid}"


@dataclass
class Cluster:
    """A synthetic cluster as integer tables.

    vals[k, i]     value id of key KEY_NAMES[k] on pod i, -1 if pod i lacks k.
    ingress[p]     policy direction (True = PolicyIngress).
    pols_off/pols_key/pols_val   CSR of the PolicySelect (podSelector) terms;
    pola_off/pola_key/pola_val   CSR of the PolicyAllow (peer) terms.
    key -1 marks the absent key (ABSENT_KEY: ABSENT_VAL).
    """
    n: int
    P: int
    mode: str
    seed: int
    vals: np.ndarray
    ingress: np.ndarray
    pols_off: np.ndarray
    pols_key: np.ndarray
    pols_val: np.ndarray
    pola_off: np.ndarray
    pola_key: np.ndarray
    pola_val: np.ndarray

    # ---- engine view -------------------------------------------------
    def working_terms(self):
        """Working selector / allow term CSRs (ingress swaps the sides,
        `kano_py/kano/model.py:82-93`); absent-key terms dropped (Q1,
        `model.py:143,146`)."""
        def pick(side_sel: bool):
            offs, keys, vals = [0], [], []
            for p in range(self.P):
                use_select = side_sel != bool(self.ingress[p])
                o, k, v = ((self.pols_off, self.pols_key, self.pols_val) if use_select
                           else (self.pola_off, self.pola_key, self.pola_val))
                for t in range(o[p], o[p + 1]):
                    if k[t] >= 0:
                        keys.append(k[t]); vals.append(v[t])
                offs.append(len(keys))
            return (np.asarray(offs, np.int64), np.asarray(keys, np.int32),
                    np.asarray(vals, np.int32))
        return pick(True), pick(False)

    def fingerprint(self) -> str:
        h = hashlib.sha256()
        for a in (self.vals, self.ingress, self.pols_off, self.pols_key, self.pols_val,
                  self.pola_off, self.pola_key, self.pola_val):
            h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest()

    # ---- object / JSON view -------------------------------------------
    def pod_labels(self, i: int) -> dict:
        d = {}
        for k in range(self.vals.shape[0]):
            v = int(self.vals[k, i])
            if v >= 0:
                d[KEY_NAMES[k]] = value_name(k, v)
        return d

    def _side(self, off, key, val, p) -> dict:
        d = {}
        for t in range(off[p], off[p + 1]):
            k = int(key[t])
            if k < 0:
                d[ABSENT_KEY] = ABSENT_VAL
            else:
                d[KEY_NAMES[k]] = value_name(k, int(val[t]))
        return d

    def to_json_obj(self) -> dict:
        pods = [{"name": f"pod{i}", "labels": self.pod_labels(i)} for i in range(self.n)]
        pols = []
        for p in range(self.P):
            pols.append({
                "name": f"pol{p}",
                "select": self._side(self.pols_off, self.pols_key, self.pols_val, p),
                "allow": self._side(self.pola_off, self.pola_key, self.pola_val, p),
                "direction": "ingress" if self.ingress[p] else "egress",
                "protocol": ["TCP", "80"],
            })
        return {"pods": pods, "policies": pols}


def make_cluster(n: int, P: int, mode: str = "sparse", seed: int = 0,
                 absent_frac: float = 0.01, **dense) -> Cluster:
    if mode == "dense":
        return make_dense(n, P, seed, absent_frac=absent_frac, **dense)
    if mode not in ("sparse", "broad"):
        raise ValueError(f"unknown mode {mode!r}")
    rng = np.random.Generator(np.random.PCG64(seed))
    n_ns = max(16, n // 1000)
    n_app = max(1, n // 20)

    ns_w = _zipf_weights(n_ns, 1.1)
    app_w = _zipf_weights(n_app, 1.3, 50.0)
    tenant_of_ns = rng.choice(N_TENANTS, size=n_ns, p=_zipf_weights(N_TENANTS, 1.2))
    ns_of_app = rng.choice(n_ns, size=n_app, p=ns_w)

    app = rng.choice(n_app, size=n, p=app_w)
    ns = ns_of_app[app]
    tenant = tenant_of_ns[ns]
    role = rng.integers(0, N_ROLES, size=n)

    nk = len(KEY_NAMES)
    vals = np.full((nk, n), -1, dtype=np.int32)
    vals[K_TENANT] = tenant
    vals[K_NS] = ns
    vals[K_APP] = app
    vals[K_ROLE] = role
    n_extra = rng.integers(0, 4, size=n)
    extra_w = _zipf_weights(N_EXTRA_VALS, 1.1)
    for slot in range(3):
        has = n_extra > slot
        idx = np.nonzero(has)[0]
        keys = rng.integers(0, N_EXTRA_KEYS, size=idx.size)
        v = rng.choice(N_EXTRA_VALS, size=idx.size, p=extra_w)
        # later slots may hit a key already set: the dict keeps one value per key
        vals[len(FIXED_KEYS) + keys, idx] = v

    ingress = rng.random(P) < 0.5
    a = rng.integers(0, n, size=P)
    b = rng.integers(0, n, size=P)
    with_role = rng.random(P) < 0.5
    allow_tenant = rng.random(P) < 0.5
    abs_s = rng.random(P) < absent_frac
    abs_a = rng.random(P) < absent_frac

    def build(side_a: bool):
        off, key, val = [0], [], []
        for p in range(P):
            pod = a[p] if side_a else b[p]
            if mode == "sparse":
                terms = [K_NS, K_APP]
                if side_a and with_role[p]:
                    terms.append(K_ROLE)
            else:
                terms = [K_NS] if (side_a or not allow_tenant[p]) else [K_TENANT]
            for k in terms:
                key.append(k); val.append(int(vals[k, pod]))
            if (abs_s[p] if side_a else abs_a[p]):
                key.append(-1); val.append(-1)
            off.append(len(key))
        return (np.asarray(off, np.int64), np.asarray(key, np.int32),
                np.asarray(val, np.int32))

    so, sk, sv = build(True)
    ao, ak, av = build(False)
    return Cluster(n, P, mode, seed, vals, ingress, so, sk, sv, ao, ak, av)


def make_dense(n: int, P: int, seed: int = 0, tenants: int = 4, apps: int = 2000,
               broad: float = 0.9, absent_frac: float = 0.01) -> Cluster:
    """The ``dense`` mode (module docstring): few uniform tenants, broad
    intra-tenant {tenant} policies plus narrow {tenant, app} ones, egress."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nk = len(KEY_NAMES)
    vals = np.full((nk, n), -1, dtype=np.int32)
    vals[K_TENANT] = rng.integers(0, tenants, size=n)
    vals[K_APP] = rng.integers(0, apps, size=n)
    vals[K_NS] = vals[K_APP] % 16
    vals[K_ROLE] = rng.integers(0, N_ROLES, size=n)
    ingress = np.zeros(P, dtype=bool)
    a = rng.integers(0, n, size=P)
    b = rng.integers(0, n, size=P)
    is_broad = rng.random(P) < broad
    abs_s = rng.random(P) < absent_frac
    abs_a = rng.random(P) < absent_frac

    def build(side_a: bool):
        off, key, val = [0], [], []
        for p in range(P):
            pod = a[p] if (side_a or is_broad[p]) else b[p]
            for k in ((K_TENANT,) if is_broad[p] else (K_TENANT, K_APP)):
                key.append(k); val.append(int(vals[k, pod]))
            if (abs_s[p] if side_a else abs_a[p]):
                key.append(-1); val.append(-1)
            off.append(len(key))
        return (np.asarray(off, np.int64), np.asarray(key, np.int32),
                np.asarray(val, np.int32))

    so, sk, sv = build(True)
    ao, ak, av = build(False)
    return Cluster(n, P, "dense", seed, vals, ingress, so, sk, sv, ao, ak, av)


def make_config(name: str) -> Cluster:
    n, P, mode, seed, *kw = CONFIGS[name]
    return make_cluster(n, P, mode, seed, **(kw[0] if kw else {}))


def cluster_objects(cl: Cluster, model_module=None):
    """Materialise the cluster as kano API objects (Container / Policy).

    ``model_module`` defaults to this package's drop-in ``kano.model``; the
    golden-vector harness passes the reference's own module instead.
    """
    if model_module is None:
        from . import model as model_module
    m = model_module
    obj = cl.to_json_obj()
    return objects_from_json(obj, m)


def objects_from_json(obj: dict, m) -> tuple:
    containers = [m.Container(p["name"], p["labels"]) for p in obj["pods"]]
    policies = []
    for q in obj["policies"]:
        d = m.PolicyIngress if q["direction"] == "ingress" else m.PolicyEgress
        allow = q["allow"]
        policies.append(m.Policy(q["name"], m.PolicySelect(q["select"]),
                                 m.PolicyAllow(allow), d,
                                 m.PolicyProtocol(q.get("protocol") or [])))
    return containers, policies


def dump_json(cl: Cluster, path: str) -> None:
    with open(path, "w") as f:
        json.dump(cl.to_json_obj(), f, separators=(",", ":"))
