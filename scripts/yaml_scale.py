"""End to end from YAML at scale: write a synthetic config as one file per
pod / policy (the reference generator's layout), then time
ConfigParser.parse + intern (the drop-in path, single core) against the bulk
front end (kano/bulk.py, process pool), and the GPU verify on the result.
Usage: python scripts/yaml_scale.py [C3] [workers] [dir]"""
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd")]
import numpy as np  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
workers = int(sys.argv[2]) if len(sys.argv) > 2 else 16
d = sys.argv[3] if len(sys.argv) > 3 else f"/tmp/kano_yaml_{cfg}"
from kano import bulk  # noqa: E402
from kano.synth import make_config  # noqa: E402
from kano.parser import ConfigParser  # noqa: E402
from kano._intern import intern  # noqa: E402

cl = make_config(cfg)
out = {"config": cfg, "pods": cl.n, "policies": cl.P, "workers": workers}
t = time.perf_counter()
out["files"] = bulk.write_cluster_yaml(cl, d)
out["write_s"] = round(time.perf_counter() - t, 2)
t = time.perf_counter()
b = bulk.load_tables(d, workers=workers, label="tenant")
out["bulk_s"] = round(time.perf_counter() - t, 2)
if cl.n <= 200_000:
    t = time.perf_counter()
    cs, ps = ConfigParser(d).parse()
    out["configparser_s"] = round(time.perf_counter() - t, 2)
    t = time.perf_counter()
    ref = intern(cs, ps)
    out["intern_s"] = round(time.perf_counter() - t, 2)
    out["tables_equal"] = all(np.array_equal(getattr(b.tables, f), getattr(ref, f))
                              for f in ("pod_val", "sel_off", "sel_col", "sel_val",
                                        "alw_off", "alw_col", "alw_val"))
if os.environ.get("KANO_YAML_GPU", "1") == "1":
    import torch  # noqa: F401
    from kano._engine import DeviceBuild
    t = time.perf_counter()
    eng = DeviceBuild(b.tables, build=False)
    eng.set_groups(b.groups)
    out["upload_s"] = round(time.perf_counter() - t, 3)
    eng.verify("stored", sys_row=0, shadow=True)          # warm
    t = time.perf_counter()
    r = eng.verify("stored", sys_row=0, shadow=True)
    out["verify_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    out["shadow_pairs"] = int(r["shadow_count"])
    out["all_isolated"] = int(len(r["all_isolated"]))
    eng.close()
print(json.dumps(out), flush=True)
if os.environ.get("KANO_YAML_KEEP") != "1":
    shutil.rmtree(d, ignore_errors=True)
