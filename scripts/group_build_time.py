"""build_matrix through the drop-in API with G members against G = 1, on the
devices KANO_DEVICES names (one device repeated = members sharing it): the
same fresh objects, the same matrix (row digests compared), the build's wall
time (median of --reps fresh builds after one warm-up), then the checks.

    KANO_DEVICES=0,0 python3 scripts/group_build_time.py [C3] [--reps 5]
"""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "kubernetes-verification_amd"))


def run(G, cl, reps):
    from kano import model, algorithm as alg
    from kano.synth import cluster_objects
    os.environ["KANO_NGPU"] = str(G)
    times, checks = [], []
    digest = None
    for r in range(reps + 1):
        cs, ps = cluster_objects(cl, model)
        t = time.perf_counter()
        m = model.ReachabilityMatrix.build_matrix(cs, ps)
        bt = time.perf_counter() - t
        t = time.perf_counter()
        res = (alg.all_reachable(m), alg.all_isolated(m), alg.user_crosscheck(m, cs, "tenant"),
               alg.system_isolation(m, 0), len(alg.policy_shadow(m, ps, cs)))
        ct = time.perf_counter() - t
        if r > 0:
            times.append(bt)
            checks.append(ct)
        key = (len(res[0]), len(res[1]), len(res[2]), len(res[3]), res[4])
        digest = digest or key
        assert key == digest, (key, digest)
        del m
    return {"G": G, "build_matrix_s": round(statistics.median(times), 4),
            "checks_s": round(statistics.median(checks), 4), "result_sizes": list(digest)}


def main():
    from kano.synth import make_config
    cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "C3"
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 5
    cl = make_config(cfg)
    devs = os.environ.get("KANO_DEVICES", "0,0")
    G = len(devs.split(","))
    one = run(1, cl, reps)
    many = run(G, cl, reps)
    assert one["result_sizes"] == many["result_sizes"]
    print(json.dumps({"config": cfg, "devices": devs, "one": one, "group": many}))
    if "--phases" in sys.argv:    # the engine's parts: create, upload, build
        from kano._engine import DeviceBuild
        from kano._intern import tables_from_cluster
        from kano.multi import MultiBuild
        tb = tables_from_cluster(cl)
        out = {}
        for g in (1, G):
            ph = []
            for _ in range(3):
                t0 = time.perf_counter()
                e = DeviceBuild(None, lean=True) if g == 1 else MultiBuild(
                    tb, g, devices=[int(x) for x in devs.split(",")], build=False, lean=True)
                t1 = time.perf_counter()
                if g == 1:
                    e.upload(tb)
                t2 = time.perf_counter()
                e.build()
                t3 = time.perf_counter()
                e.close()
                ph.append((t1 - t0, t2 - t1, t3 - t2))
            out[g] = [round(statistics.median(x[k] for x in ph), 4) for k in range(3)]
        print(json.dumps({"phases_create_upload_build_s": out}))
    if "--profile" in sys.argv:   # where a G-member build_matrix spends its time
        import cProfile
        import pstats
        from kano import model
        from kano.synth import cluster_objects
        for g in (1, G):
            os.environ["KANO_NGPU"] = str(g)
            cs, ps = cluster_objects(cl, model)
            pr = cProfile.Profile()
            pr.enable()
            m = model.ReachabilityMatrix.build_matrix(cs, ps)
            pr.disable()
            print(f"== G={g}", file=sys.stderr)
            pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(10)
            del m


if __name__ == "__main__":
    main()
