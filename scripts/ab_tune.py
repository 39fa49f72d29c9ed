"""A/B of KANO_TUNE settings on one box: bench.py lines alternated, summary.

    python scripts/ab_tune.py --config C3 --steps 300 --reps 2 -- "" "store=2" ...

A setting is "TUNE" or "LIB|TUNE" (LIB: a libkano_hip.so to load through
KANO_HIP_LIB, e.g. a baseline build, paths relative to the repo).  Each setting runs as its own bench.py process (timeout-bounded), in turn,
`reps` times; prints one summary line per run and writes the JSON lines to
gpurun_out/ab_<config>.jsonl."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--extra", default="")
    ap.add_argument("--timeout", type=int, default=150)
    ap.add_argument("tunes", nargs="*")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", f"ab_{a.config}.jsonl"), "a")
    for rep in range(a.reps):
        for t in a.tunes or [""]:
            lib, _, tune = t.rpartition("|")
            env = dict(os.environ, KANO_TUNE=tune)
            if lib:
                env["KANO_HIP_LIB"] = os.path.join(ROOT, lib)
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", a.config,
                   "--steps", str(a.steps), "--warmup", str(a.warmup), "--cpu-baseline", "0",
                   "--cold", "0"] + a.extra.split()
            r = subprocess.run(["timeout", "-k", "10", str(a.timeout)] + cmd, env=env,
                               capture_output=True, text=True, cwd=ROOT)
            if r.returncode != 0:
                print(f"[{t}] rc={r.returncode}\n{r.stdout[-1500:]}\n{r.stderr[-3000:]}", flush=True)
                sys.exit(r.returncode)
            line = json.loads(r.stdout.strip().splitlines()[-1])
            line["tune"] = t
            out.write(json.dumps(line) + "\n")
            out.flush()
            rf = line.get("roofline") or {}
            al = rf.get("alone") or {}
            mr = line.get("mfma_roofline") or {}
            print(f"rep {rep} [{t or 'default'}] mean {line['ms_per_step']:.4f} median "
                  f"{line['step_ms']['median']:.4f} k_rows {rf.get('avg_launch_ms', 0):.4f} "
                  f"(frac {rf.get('frac', 0):.3f}) alone {al.get('avg_launch_ms', 0) or 0:.4f} "
                  f"(frac {al.get('frac', 0) or 0:.3f}) mfma {mr.get('frac', '-')} "
                  f"verified {line.get('verified')}", flush=True)


if __name__ == "__main__":
    main()
