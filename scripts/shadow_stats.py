"""policy_shadow candidate statistics on a synthetic config: |S(c)| per row
class, the candidate pairs sum_c s_c^2 and how many distinct (j, k) policy
pairs they hold (how much a per-pair dedup would save).
Usage: python scripts/shadow_stats.py [C3] [rank_of]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd")]
import torch  # noqa: E402,F401
import numpy as np  # noqa: E402
from kano._engine import DeviceBuild  # noqa: E402
from kano._intern import tables_from_cluster  # noqa: E402
from kano.synth import make_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
rank_of = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cl = make_config(cfg)
n = cl.n
eng = DeviceBuild(tables_from_cluster(cl), rows=(0, n // rank_of))
off, pol = eng.select_csr()
s = np.diff(off)
print(f"{cfg} rows 0..{n // rank_of}: classes {len(s)}, sum s {s.sum()}, sum s^2 {(s.astype(np.int64) ** 2).sum()}")
for q in (50, 90, 99, 99.9, 100):
    print(f"  s p{q}: {np.percentile(s, q):.0f}")
big = np.argsort(s)[-10:][::-1]
print("  largest s:", s[big].tolist())
pairs = set()
tot = 0
for c in range(len(s)):
    L = pol[off[c]:off[c + 1]]
    if len(L) < 2:
        continue
    a = np.repeat(L, len(L)).astype(np.int64)
    b = np.tile(L, len(L)).astype(np.int64)
    k = a * 1_000_000 + b
    tot += len(k)
    pairs.update(k.tolist())
print(f"  candidate pairs {tot}, distinct (j,k) {len(pairs)}")
eng.close()
