"""Multi-hop reachability across row shards (SURVEY.md §8(e) + §8(f) rank 3):
each rank builds its rows, writes its part of the one-hop table T
(kano_path_shard), one RCCL all-gather over xGMI collects the parts, and
kano_path_combine writes the rank's rows of the path matrix.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        scripts/path_dist.py --config C3 [--hops 2]
    python scripts/path_dist.py --config C5 --emulate 8    # rank 0 of 8 on one GPU

--emulate N builds every shard on this GPU in turn (keeping only rank 0's),
fills the gathered buffer with a local copy and times rank 0's steps.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--hops", type=int, default=2)
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--emulate", type=int, default=0)
    a = ap.parse_args()
    import torch
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.shard import row_range
    from kano.synth import make_config
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if a.emulate == 0 and "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    N = a.emulate or world
    cl = make_config(a.config)
    t = tables_from_cluster(cl)
    n = cl.n
    r0, r1 = row_range(n, N, rank if not a.emulate else 0)
    t0 = time.perf_counter()
    eng = DeviceBuild(t, rows=(r0, r1))
    nw = eng.path_shard_words()
    gathered = torch.zeros(N * max(nw, 1), dtype=torch.int64, device="cuda")
    part = torch.zeros(max(nw, 1), dtype=torch.int64, device="cuda")
    if a.emulate:
        for k in range(1, N):        # the other ranks' parts, built in turn
            e = DeviceBuild(t, rows=row_range(n, N, k))
            e.path_shard(gathered.data_ptr() + 8 * nw * k)
            e.close()
    dst = DeviceBuild.empty(n, rows=(r0, r1))
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    times = []
    info = None
    for _ in range(a.reps):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        eng.path_shard(part.data_ptr())
        s1 = time.perf_counter()
        if dist:
            dist.all_gather_into_tensor(gathered, part)
        else:
            gathered[:nw].copy_(part[:nw])
        torch.cuda.synchronize()
        s2 = time.perf_counter()
        info = dst.path_combine(eng, gathered.data_ptr(), N, a.hops, a.mode)
        s3 = time.perf_counter()
        times.append((s1 - s0, s2 - s1, s3 - s2, s3 - s0))
    best = min(times, key=lambda x: x[3])
    if dist:
        tt = torch.tensor([best[3]], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        total = float(tt.item())
    else:
        total = best[3]
    if rank == 0:
        print(json.dumps({
            "config": a.config, "n": n, "hops": a.hops, "ranks": N,
            "emulated": bool(a.emulate), "rows": [r0, r1], "T_words": nw,
            "ms": {"shard_T": round(best[0] * 1e3, 3), "gather": round(best[1] * 1e3, 3),
                   "combine_steps_expand": round(best[2] * 1e3, 3),
                   "total_max_over_ranks": round(total * 1e3, 3)},
            "gathered_MB": round(N * nw * 8 / 1e6, 1), "info": info,
            "setup_s": round(t_setup, 2)}), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
