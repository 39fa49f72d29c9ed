"""Where the drop-in's cold time goes: build_matrix on fresh C3 objects, then
the five checks through kano.algorithm, each under cProfile (top functions by
internal time), after one unprofiled warm-up round (GPU runtime up).

    python3 scripts/cold_profile.py [C3] [--top 12]
"""
import cProfile
import io
import os
import pstats
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "kubernetes-verification_amd"))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "C3"
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    from kano import model, algorithm as alg
    from kano.synth import make_config, cluster_objects
    cl = make_config(cfg)
    steps = [("build_matrix", lambda s: s.update(m=model.ReachabilityMatrix.build_matrix(s["cs"], s["ps"]))),
             ("all_reachable", lambda s: alg.all_reachable(s["m"])),
             ("all_isolated", lambda s: alg.all_isolated(s["m"])),
             ("user_crosscheck", lambda s: alg.user_crosscheck(s["m"], s["cs"], "tenant")),
             ("system_isolation", lambda s: alg.system_isolation(s["m"], 0)),
             ("policy_shadow", lambda s: alg.policy_shadow(s["m"], s["ps"], s["cs"]))]
    plain = {}
    for rnd in range(3):   # warm-up, timed, profiled: fresh objects each round
        cs, ps = cluster_objects(cl, model)
        st = {"cs": cs, "ps": ps}
        for name, fn in steps:
            if rnd < 2:
                t = time.perf_counter()
                fn(st)
                plain[name] = time.perf_counter() - t
                continue
            pr = cProfile.Profile()
            pr.enable()
            fn(st)
            pr.disable()
            out = io.StringIO()
            pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(top)
            print(f"== {name}: {plain[name] * 1e3:.1f} ms unprofiled", flush=True)
            print("\n".join(l for l in out.getvalue().splitlines()[6:] if l.strip()), flush=True)
        st["m"].engine.close()


if __name__ == "__main__":
    main()
