"""How many of a row shard's classes share their select list S(c), and what
share of policy_shadow's candidate pairs (sum |S(c)|^2 over classes with local
members) the duplicates carry: the case for testing each distinct list once.
Usage: python scripts/shadow_dup_stats.py CONFIG NSHARDS"""
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
U = off.shape[0] - 1
mc = np.bincount(cls, minlength=U)
seen = {}
tot = dup = 0
ndup = nlive = 0
for c in range(U):
    s = off[c + 1] - off[c]
    if mc[c] == 0 or s == 0:
        continue
    nlive += 1
    key = pol[off[c]:off[c + 1]].tobytes()
    w = int(s) * int(s)
    tot += w
    if key in seen:
        dup += w
        ndup += 1
    else:
        seen[key] = c
print(f"{cfg} rows [0, {n // N}): classes {U}, with members and S {nlive}, distinct lists "
      f"{len(seen)}, duplicate classes {ndup}; candidate pairs {tot:.3e}, on duplicates "
      f"{dup:.3e} ({100.0 * dup / max(tot, 1):.1f} %)")
e.close()
