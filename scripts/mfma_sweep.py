"""The dense path's crossover: the heavy classes' Mc rows by the bitwise OR
(k_heavy_mc_or, reads ldMc words per (heavy class, policy in S(c))) against
the fp4 MFMA GEMM (k_heavy_gemm_f4, 2 H P Ua ops whatever the density) and the
split-K MFMA kernel (k_heavy_mc_mfma), on `dense` clusters (kano/synth.py)
whose selector density broad/tenants is swept at a fixed class count.

One JSON line per cluster: the class counts, the heavy classes' selector
density, every variant's contraction time (HIP events around the kernel,
kano_mfma_timing), its rate, the whole build's wall time, and whether every
variant wrote the same matrix (row digests).  AUTO's choice is run last and
reported with the variant it picked.

    python3 scripts/mfma_sweep.py [--n 100000] [--P 10000] [--reps 5] [--quick]
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-verification_amd"))

VARIANTS = [("bitwise", "bitwise", "hortime=1"), ("gemm22", "mfma", "hgemm=22"),
            ("gemm42", "mfma", "hgemm=42"), ("gemm44", "mfma", "hgemm=44"),
            ("splitk", "mfma", "hgemm=0"), ("auto", "auto", "hortime=1")]


def run_point(tb, n, reps, variants):
    from kano._engine import DeviceBuild
    out, digests = {}, {}
    for name, path, tune in variants:
        os.environ["KANO_TUNE"] = tune
        eng = DeviceBuild(tb, build=False, path=path)
        eng.build()                                  # warm (allocations)
        eng.mfma_timing(reset=True)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.build()
        wall = (time.perf_counter() - t0) / reps * 1e3
        mt = eng.mfma_timing()
        info = eng.info()
        digests[name] = hashlib.sha256(eng.rows_digest(0, n).tobytes()).hexdigest()
        ms = mt["sum_ms"] / mt["builds"] if mt["builds"] else None
        out[name] = {"contraction_ms": round(ms, 4) if ms else None,
                     "tops": round(mt["ops_last"] / (ms * 1e-3) / 1e12, 1) if ms else None,
                     "build_ms": round(wall, 3), "heavy_path": info["HEAVY_PATH"]}
        if name == "auto":
            base = dict(U=info["U"], H=info["HEAVY"], Ua=info["UA"], nnz_sel=info["NNZ_SEL"],
                        heavy_sel=info["HEAVY_SEL"],
                        ops=mt["ops_last"])
        eng.close()
    os.environ["KANO_TUNE"] = ""
    agree = len(set(digests.values())) == 1
    return base, out, agree


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--P", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--quick", action="store_true", help="three points, two variants")
    a = ap.parse_args()
    from kano._intern import tables_from_cluster
    from kano.synth import make_cluster
    # (tenants, apps, broad): density ~ broad / tenants at ~8,000 row and
    # column classes, then the class count itself
    points = [(4, 2000, b) for b in (0.01, 0.02, 0.05, 0.1, 0.2, 0.4, 0.9)] + \
             [(8, 1000, 0.9), (16, 500, 0.9), (2, 2000, 0.9), (4, 500, 0.9), (4, 4000, 0.9)]
    variants = VARIANTS
    if a.quick:
        points = [(4, 2000, 0.02), (4, 2000, 0.2), (4, 2000, 0.9)]
        variants = [v for v in VARIANTS if v[0] in ("bitwise", "gemm22", "gemm44",
                                                     "auto")]
    for T, A, b in points:
        t0 = time.perf_counter()
        cl = make_cluster(a.n, a.P, "dense", seed=4, tenants=T, apps=A, broad=b)
        tb = tables_from_cluster(cl)
        base, res, agree = run_point(tb, a.n, a.reps, variants)
        H = max(1, base["H"])
        line = {"tenants": T, "apps": A, "broad": b, "n": a.n, "P": a.P, **base,
                "sel_density_est": round(b / T, 4), "agree": agree, "variants": res,
                "secs": round(time.perf_counter() - t0, 1)}
        print(json.dumps(line), flush=True)
        print(f"T={T} A={A} b={b}: H={H} " + " ".join(
            f"{k}={v['contraction_ms']}" for k, v in res.items()), file=sys.stderr, flush=True)
        if not agree:
            print("variants disagree", file=sys.stderr)
            sys.exit(1)


if __name__ == "__main__":
    main()
