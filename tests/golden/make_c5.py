"""Expected outputs for the C5 benchmark cluster (10^6 pods, 10^5 policies),
which kano_py cannot run (its matrix is 10^6 bitarrays of 10^6 bits and
policy_shadow loops over ~10^11 tuples), and for D1, the dense-path cluster
(10^5 pods, 10^4 policies, 8,000 row classes each selected by ~2,250
policies; kano_py's policy_shadow would loop over ~10^12 tuples):

    python3 tests/golden/make_c5.py            # repo python, ~2-4 min, ~10 GB RAM
    python3 tests/golden/make_c5.py D1         # ~3 min

The outputs come from oracle/kano_indexed.py, an indexed restatement of
kano_py's build_matrix and checks that shares no code with the product and is
pinned against kano_py's own records on C2, C3 and C4 (every check list, the
matrix sha256, the select / allow set and list shas, policy_shadow's pairs
sha256 or C4's count; tests/test_oracle_indexed.py).  Written to
tests/golden/expected/C5.json in make_golden.py's layout (long index lists as
count + sha256 + head), plus:

* ``row_digests_sha256``  sha256 of kano_rows_digest over all 10^6 rows
  (uint64 little-endian, pod order) -- every bit of the 125 GB matrix under
  the digest;
* ``row_digest_sample``   512 seeded rows and their digests (hex).
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-verification_amd"))

from kano.synth import CONFIGS, K_TENANT, make_config  # noqa: E402  (the input generator)
from oracle import kano_indexed as K  # noqa: E402


def record(name: str, log=print) -> dict:
    t0 = time.time()
    cl = make_config(name)
    ix = K.build_cluster(cl, label_key=K_TENANT)
    log(f"{name}: {ix.size.shape[0]} classes, R nnz {ix.R.nnz}  ({time.time() - t0:.1f} s)")
    RT = K.column_classes(ix)
    rec = {"name": name, "label": "tenant",
           "seed": {"n": cl.n, "P": cl.P, "mode": cl.mode, "seed": cl.seed,
                    "fingerprint": cl.fingerprint()},
           "n": cl.n, "P": cl.P,
           "source": "tests/golden/make_c5.py (oracle/kano_indexed.py, pinned on C2/C3/C4 "
                     "against kano_py's records)"}
    rec["all_reachable"] = K.list_record(K.all_reachable(ix, RT))
    rec["all_isolated"] = K.list_record(K.all_isolated(ix, RT))
    rec["user_crosscheck"] = {"label": "tenant", "result": K.list_record(K.user_crosscheck(ix, RT))}
    rec["system_isolation"] = {"idx": 0, "result": K.list_record(K.system_isolation(ix, 0))}
    log(f"lists ({time.time() - t0:.1f} s)")
    if name == "D1":
        # (~5e11 pairs: the count alone, every pair's subset test counted)
        cnt, _ = K.policy_shadow(ix, want_sha=False)
        rec["policy_shadow"] = {"count": cnt}
    else:
        cnt, sh = K.policy_shadow(ix)
        rec["policy_shadow"] = {"count": cnt, "sha256": sh}
    log(f"policy_shadow {cnt} ({time.time() - t0:.1f} s)")
    dig = K.row_digests(ix)
    rec["row_digests_sha256"] = hashlib.sha256(dig.astype("<u8").tobytes()).hexdigest()
    rng = np.random.default_rng(55)
    rows = np.unique(np.concatenate([[0, cl.n - 1], rng.integers(0, cl.n, 510)]))
    rec["row_digest_sample"] = {"rows": rows.tolist(), "digest": [f"{int(d):016x}" for d in dig[rows]]}
    ones = int((ix.R @ ix.size)[ix.cls].sum())
    rec["density"] = ones / max(1, cl.n * cl.n)
    log(f"digests, density {rec['density']:.3g} ({time.time() - t0:.1f} s)")
    return rec


def main():
    names = sys.argv[1:] or ["C5"]
    for name in names:
        assert name in CONFIGS, name
        rec = record(name)
        path = os.path.join(HERE, "expected", f"{name}.json")
        if name not in ("C5", "D1"):
            path = os.path.join("/tmp", f"{name}_indexed.json")   # C2-C4 hold kano_py's own
        with open(path, "w") as f:
            json.dump(rec, f, separators=(",", ":"))
        print("wrote", path)


if __name__ == "__main__":
    main()
