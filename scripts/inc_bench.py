"""Incremental policy updates on a BASELINE config:
time kano_add_policies / kano_remove_policies of one policy against a full
rebuild, engine level (interned tables resident in HBM) and through the
drop-in API (ReachabilityMatrix.add_policies / remove_policies, including the
host-side list bookkeeping).  Prints one JSON line.

    python scripts/inc_bench.py [--config C3] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from kano import model
    from kano._engine import DeviceBuild
    from kano._intern import intern, intern_more
    from kano.synth import make_config, objects_from_json
    cl = make_config(a.config)
    obj = cl.to_json_obj()
    cs, ps = objects_from_json(obj, model)
    P = len(ps)
    base, extra = ps[:P - a.reps], ps[P - a.reps:]
    t0 = time.perf_counter()
    tables = intern(cs, base)
    t_intern = time.perf_counter() - t0
    eng = DeviceBuild(tables)
    # full rebuild, engine level (tables resident)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        eng.build()
        eng.rows(0, 1)
        ts.append(time.perf_counter() - t0)
    t_build = min(ts)
    # add one policy at a time, engine level
    adds, rems, sizes = [], [], []
    for pol in extra:
        x, s, al = intern_more(tables, [pol])
        t0 = time.perf_counter()
        eid = eng.add_policies(x, s, al)
        adds.append(time.perf_counter() - t0)
        sw, aw = eng.added_policy_sets(eid)
        sizes.append(int(np.unpackbits(sw.view(np.uint8)).sum()))
    for k in range(a.reps):
        t0 = time.perf_counter()
        eng.remove_policies([k * 7])
        rems.append(time.perf_counter() - t0)
    # the drop-in API: a build over base, then add / remove through the matrix
    m = model.ReachabilityMatrix.build_matrix(cs, base)
    _ = cs[0].select_policies          # materialise the build's lists
    t0 = time.perf_counter()
    m.add_policies(extra[:1])
    t_api_add = time.perf_counter() - t0
    t0 = time.perf_counter()
    m.remove_policies([3])
    t_api_rem = time.perf_counter() - t0
    out = {"config": a.config, "n": cl.n, "P": P,
           "engine_build_ms": round(t_build * 1e3, 3),
           "engine_add_one_ms": [round(t * 1e3, 3) for t in adds],
           "added_sel_rows": sizes,
           "engine_remove_one_ms": [round(t * 1e3, 3) for t in rems],
           "api_add_one_ms": round(t_api_add * 1e3, 3),
           "api_remove_one_ms": round(t_api_rem * 1e3, 3),
           "host_intern_full_s": round(t_intern, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
