"""policy_shadow's candidate pairs by class on a row shard: the largest
|S(c)| classes, and how many distinct allow sets their policies have (the
case for testing per pair of allow-set groups instead of per pair of
policies).  Usage: python scripts/shadow_group_stats.py CONFIG NSHARDS"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd")]
from kano._engine import DeviceBuild  # noqa: E402
from kano._intern import tables_from_cluster  # noqa: E402
from kano.synth import make_config  # noqa: E402

cfg, N = sys.argv[1], int(sys.argv[2])
cl = make_config(cfg)
n = cl.n
e = DeviceBuild(tables_from_cluster(cl), rows=(0, n // N))
cls = e.classes()[: n // N]
off, pol = e.select_csr()
aoff, apods = e.allow_csr()
P = aoff.shape[0] - 1
U = off.shape[0] - 1
mc = np.bincount(cls, minlength=U)
# allow-set group of every policy (hash of its allowed-pod list)
gid = np.empty(P, np.int64)
seen = {}
for p in range(P):
    h = hashlib.blake2b(apods[aoff[p]:aoff[p + 1]].tobytes(), digest_size=16).digest()
    gid[p] = seen.setdefault(h, len(seen))
print(f"{cfg} shard 0 of {N}: P {P}, distinct allow sets {len(seen)}")
sz = np.diff(off)
live = (mc > 0) & (sz > 0)
w = np.where(live, sz.astype(np.int64) ** 2, 0)
order = np.argsort(-w)
tot = w.sum()
acc = 0
for c in order[:15]:
    s = pol[off[c]:off[c + 1]]
    g = np.unique(gid[s]).shape[0]
    acc += w[c]
    print(f"  class {c}: members {mc[c]}, |S| {sz[c]}, pairs {w[c]:.3e} ({100.0 * acc / tot:.1f} % "
          f"cumulative), distinct allow sets in S {g} -> group pairs {g * g:.3e}")
e.close()
