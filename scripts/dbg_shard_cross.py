"""Debug: per-shard user_crosscheck on C2 against the shard's own rows of M,
through kano_verify and through kano_verify_shard's gathered words."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd")]
import torch  # noqa: E402
import numpy as np  # noqa: E402
from kano._engine import DeviceBuild  # noqa: E402
from kano._intern import tables_from_cluster  # noqa: E402
from kano._bits import words_to_bool  # noqa: E402
from kano.synth import make_config, KEY_NAMES  # noqa: E402

cl = make_config("C2")
t = tables_from_cluster(cl)
n = cl.n
W = (n + 63) // 64
gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
spans = [(k * n // N, (k + 1) * n // N) for k in range(N)]
gathered = torch.zeros(N * 3 * W, dtype=torch.int64, device="cuda")
engs = [DeviceBuild(t, rows=s, build=False) for s in spans]
seq = len(sys.argv) > 2
for k, e in enumerate(engs):
    e.verify_shard(gathered.data_ptr() + 8 * 3 * W * k, gid=gid, sys_row=0, shadow=False)
    if seq:
        torch.cuda.synchronize()
torch.cuda.synchronize()
g = gathered.cpu().numpy().view(np.uint64).reshape(N, 3, W)
full = np.zeros(n, bool)
for k, (e, (r0, r1)) in enumerate(zip(engs, spans)):
    M = np.stack([words_to_bool(w, n) for w in e.rows(r0, r1 - r0)])
    truth = np.zeros(n, bool)
    for q, i in enumerate(range(r0, r1)):
        truth |= M[q] & (gid != gid[i])
    full |= truth
    got = words_to_bool(g[k, 1], n)
    bad = np.flatnonzero(got != truth)
    print(f"shard {k} words: cross {got.sum()} truth {truth.sum()} bad {len(bad)} "
          f"{bad[:10].tolist()} got_at_bad {got[bad[:10]].astype(int).tolist()}", flush=True)
r = engs[0].verify_combine(gathered.data_ptr(), N)
gotc = np.zeros(n, bool)
gotc[r["user_crosscheck"]] = True
print("combined", gotc.sum(), "truth", full.sum(), "bad", np.flatnonzero(gotc != full)[:10].tolist())
