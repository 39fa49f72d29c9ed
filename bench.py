"""Benchmark: reachability build + all Kano checks on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

One step = one pass of the hot path over the synthetic cluster, inputs
(interned label tables) already resident in HBM:
  ReachabilityMatrix.build_matrix   classes, selector evaluation, allow sets,
                                    matrix rows (kano_py/kano/model.py:125-165)
  all_reachable, all_isolated       algorithm.py:4-17
  user_crosscheck(label="tenant")   algorithm.py:27-42 (gid array uploaded)
  system_isolation(idx=0)           algorithm.py:45-55
  policy_shadow                     algorithm.py:58-80 (pairs copied to host)
with every result on the host as index arrays.  value = n^2 / step time
(pod-pairs/s); the n x n matrix is built once per step over
all ranks.  For N > 1 the rows are partitioned across ranks (one process per
GPU, kano_verify_shard); the column checks combine the ranks' [OR | cross |
NAND] bit words (3 * W u64 each) gathered by one RCCL all-gather over xGMI and
OR-ed on the device (kano_verify_combine; RCCL has no bitwise reduction);
strong scaling (fixed cluster).

Rank 0 prints ONE JSON line.  roofline: the dominant kernel is k_rows (the
matrix write), algorithmic bytes = 8 * rows * W (the bit matrix it writes),
timed with HIP events recorded by its own dispatch on its stream.
cpu_baseline: kano_py's algorithm over the WHOLE cluster (oracle/kano_cpu.c,
OpenMP, on every host thread the process gets; its outputs checked against
kano_py's record before the time counts), measured, not extrapolated.

--gpus N > 1 without torch.distributed.run runs the N row shards as members of
one kano_group in this process (KANO_DEVICES=0,0 puts two members on one
device: the exchange is then device copies).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "kubernetes-verification_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "pod-pairs/sec for reachability build + all-checks latency, 100k pods, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_I8_PEAK_TOPS = 5000.0     # MI355X_MICROARCH.md: int8 MFMA 2x the BF16 rate (~2.5 PF dense)
MFMA_F4_PEAK_TOPS = 10000.0    # MI355X_MICROARCH.md: block-scaled fp4 4x the BF16 rate (~10 PF dense)
WORKLOADS = {
    "C2": "Synthetic 10k pods / 1k policies, Zipf labels (BASELINE configs[1])",
    "C3": "Synthetic 100k pods / 10k policies, sparse selectors (BASELINE configs[2])",
    "C4": "Synthetic 100k pods / 10k policies, broad namespace-wide selectors (BASELINE configs[3])",
    "C5": "Synthetic 1M pods / 100k policies, sparse selectors (BASELINE configs[4])",
    "D1": "Synthetic 100k pods / 10k policies, dense selectors (4 tenants, 2,000 apps; the "
          "MFMA path's line, not a BASELINE config)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (many short steps: the boxes show a 7-8 ms host stall about every 0.5 s
    # of wall time inside an engine call -- no HIP call spans it, the thread
    # is off the CPU; over 1000 steps it adds 1-3% to the mean, see median)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="C3", choices=sorted(WORKLOADS))
    ap.add_argument("--path", default="auto", choices=["auto", "bitwise", "mfma"])
    ap.add_argument("--shadow", default="auto", choices=["auto", "pairs", "count", "off"],
                    help="policy_shadow: the pairs to the host (C2/C3/C5), the count only "
                         "(every subset test, no emission: C4's ~1e11 pairs), or off; "
                         "auto = count for C4, pairs otherwise")
    ap.add_argument("--no-shadow", action="store_true", help="same as --shadow off")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cold", type=int, default=1,
                    help="also time the drop-in API once on fresh objects (C2 / C3, one rank)")
    ap.add_argument("--shard-path", action="store_true",
                    help="diagnostic: the N > 1 step (shard verify + RCCL all-gather + combine) "
                         "even at one rank, e.g. under torch.distributed.run --nproc-per-node 1")
    ap.add_argument("--alone", type=int, default=5,
                    help="k_rows launches timed alone (kano_build) after the timed region "
                         "(roofline.alone; 0: none)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="kano_set_pipeline: each step queues the next step's prologue behind a "
                         "gate the next step opens (0: off)")
    ap.add_argument("--gather1", action="store_true",
                    help="diagnostic: the one-rank step through kano_verify_gather (the "
                         "emulated exchange, a device copy) instead of the fused kano_verify")
    ap.add_argument("--rank-of", type=int, default=0,
                    help="diagnostic: time rank 0's shard step of an N-rank run on one GPU "
                         "(the all-gather replaced by a local copy; not a bench line)")
    return ap.parse_args()


class Step:
    """The hot path on this rank's row shard."""

    def __init__(self, eng, gid, n, rank, world, r0, r1, shadow, dist=None, torch=None,
                 stream=None, emulate=0):
        self.eng, self.gid, self.n = eng, gid, n
        self.rank, self.world, self.r0, self.r1 = rank, world, r0, r1
        self.shadow = shadow != "off"
        self.count_only = shadow == "count"
        self.dist, self.torch, self.stream = dist, torch, stream
        self.W = (n + 63) >> 6
        self.emulate = emulate
        self.nranks = emulate or world
        self.shard_path = self.nranks > 1 or dist is not None
        if self.shard_path:
            # [OR | cross | NAND] words of this rank's rows, all ranks'
            # gathered, the combine (kano/shard.py)
            from kano.shard import ShardExchange
            self.xchg = ShardExchange(torch, self.W, self.nranks,
                                      dist=None if emulate else dist, stream=stream)
        from kano._engine import PinnedBuffer
        self.pin = None
        self.pin_idx = None
        # the tenant groups are resident input, uploaded once like the label
        # tables (user_hashmap, algorithm.py:20-24)
        eng.set_groups(gid)
        self.pin_pairs = 0
        self.PinnedBuffer = PinnedBuffer
        self.results = {}
        self.verify_max_ms = 0.0    # the slowest engine call (host hiccups show here or not)
        self.gather1 = False

    def __call__(self):
        eng, n = self.eng, self.n
        res = {}
        pairs = None
        if self.shadow and not self.count_only:
            if self.pin is None:
                self.pin_pairs = 1 << 20
                self.pin = self.PinnedBuffer(self.pin_pairs * 8)
                self.pairs_view = self.pin.view(np.int32, 2 * self.pin_pairs)
            pairs = self.pairs_view
        if self.pin_idx is None:
            self.pin_idx = self.PinnedBuffer(4 * 4 * max(n, 1))
            self.idx_view = self.pin_idx.view(np.int32, 4 * max(n, 1))
        idx = self.idx_view
        tv = time.perf_counter()
        if self.gather1:
            # (diagnostic: the same step through the gathered tail, one rank)
            r = eng.verify_gather(0, 1, gid="stored", sys_row=0, shadow=self.shadow,
                                  shadow_count_only=self.count_only, pairs=pairs, idx=idx)
        elif not self.shard_path:
            # the fused entry point: build + every check, three host syncs;
            # results arrive as the reference's index lists
            r = eng.verify("stored", sys_row=0, shadow=self.shadow, pairs=pairs, idx=idx,
                           shadow_count_only=self.count_only)
        else:
            # this rank's rows and checks up to its column words, one RCCL
            # all-gather of 3*W words per rank over xGMI (on the engine's
            # stream), then the OR-combine and the lists on the device
            r = self.xchg.verify(eng, gid="stored", sys_row=0, shadow=self.shadow,
                                 count_only=self.count_only, pairs=pairs, idx=idx)
        dv = time.perf_counter() - tv
        self.verify_max_ms = max(self.verify_max_ms, dv * 1e3)
        for k in ("all_reachable", "all_isolated", "user_crosscheck", "system_isolation"):
            if r[k] is not None:
                res[k] = r[k]
        if self.shadow:
            cnt = r["shadow_count"]
            res["policy_shadow"] = r["pairs"]
            res["policy_shadow_count"] = cnt
            if not self.count_only and cnt > self.pin_pairs:   # grow for the next step
                self.pin.close()
                self.pin_pairs = 2 * cnt
                self.pin = self.PinnedBuffer(self.pin_pairs * 8)
                self.pairs_view = self.pin.view(np.int32, 2 * self.pin_pairs)
        self.results = res
        return res


def cold_drop_in(cl, config):
    """The drop-in call a kano_py user makes once, on fresh objects, timed end
    to end (outside the bench's timed region; the process's GPU runtime is
    already up): ReachabilityMatrix.build_matrix(containers, policies) --
    interning, context, upload, build (kano_py/kano/model.py:125-165) -- then
    the five checks' lists through kano.algorithm (algorithm.py:4-80)."""
    from kano import model, algorithm as alg
    from kano.synth import cluster_objects
    t = time.perf_counter()
    cs, ps = cluster_objects(cl, model)
    t_objects = time.perf_counter() - t
    sec = {}
    t = time.perf_counter()
    m = model.ReachabilityMatrix.build_matrix(cs, ps)
    m.engine.info()                   # the build has run (kano_build syncs on its own)
    sec["build_matrix"] = time.perf_counter() - t
    t0 = time.perf_counter()
    res = {}
    for name, fn in (("all_reachable", lambda: alg.all_reachable(m)),
                     ("all_isolated", lambda: alg.all_isolated(m)),
                     ("user_crosscheck", lambda: alg.user_crosscheck(m, cs, "tenant")),
                     ("system_isolation", lambda: alg.system_isolation(m, 0)),
                     ("policy_shadow", lambda: alg.policy_shadow(m, ps, cs))):
        t = time.perf_counter()
        res[name] = fn()
        sec[name] = time.perf_counter() - t
    sec["checks_total"] = time.perf_counter() - t0
    total = sec["build_matrix"] + sec["checks_total"]
    pairs = np.array(res.pop("policy_shadow"), np.int32).reshape(-1, 2)
    res = {k: np.asarray(v, np.int32) for k, v in res.items()}
    res["policy_shadow"] = pairs
    res["policy_shadow_count"] = int(pairs.shape[0])
    verified, _ = verify_against_golden(config, cl, res, 1, 0, 0, "pairs")
    m.engine.close()
    del m, cs, ps
    # the same build_matrix in its parts, on fresh objects: host interning,
    # context creation, upload of the tables, the first build (allocations
    # included) and a second one (the steady state), the groups of
    # user_crosscheck
    from kano._engine import DeviceBuild
    from kano._intern import intern, group_ids
    cs, ps = cluster_objects(cl, model)
    parts = {}
    t = time.perf_counter()
    tb = intern(cs, ps)
    parts["intern"] = time.perf_counter() - t
    t = time.perf_counter()
    eng = DeviceBuild(None, lean=True)        # (what build_matrix creates)
    parts["context"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.upload(tb)
    parts["upload"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.build()
    parts["first_build"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.build()
    parts["second_build"] = time.perf_counter() - t
    t = time.perf_counter()
    group_ids(cs, "tenant")
    parts["group_ids"] = time.perf_counter() - t
    eng.close()
    return {"seconds": {k: round(v, 4) for k, v in sec.items()}, "total_s": round(total, 4),
            "build_matrix_parts_s": {k: round(v, 4) for k, v in parts.items()},
            "objects_s": round(t_objects, 3), "verified": verified,
            "note": "build_matrix on fresh Container / Policy objects, then all_reachable, "
                    "all_isolated, user_crosscheck(tenant), system_isolation(0), policy_shadow "
                    "through the drop-in API (lists as Python objects); the GPU runtime is "
                    "already initialised; objects_s (creating the objects) is not included"}


def _cpu_lib():
    import ctypes
    path = os.path.join(ROOT, "oracle", "libkano_cpu.so")
    L = ctypes.CDLL(path)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    L.cpu_threads.argtypes = [i32]
    L.cpu_build.argtypes = [i64, i64, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.cpu_col_reduce.argtypes = [i64, vp, i32, vp]
    L.cpu_crosscheck.argtypes = [i64, vp, vp, vp]
    L.cpu_lists.argtypes = [i64, i64, vp, vp, vp]
    L.cpu_shadow.argtypes = [i64, i64, vp, vp, vp, i64, vp, ctypes.POINTER(i64)]
    return L


def cpu_baseline(cl, gid, config):
    """The reference's algorithm (kano_py: build_matrix, all_reachable,
    all_isolated, user_crosscheck, system_isolation, policy_shadow) over the
    WHOLE cluster on the host's cores (oracle/kano_cpu.c, OpenMP; the same
    per-element work as the single-threaded oracle/kano_oracle.c restatement),
    timed end to end and checked against kano_py's record of the cluster."""
    import ctypes
    import hashlib
    L = _cpu_lib()
    n, P = cl.n, cl.P
    p = lambda a: a.ctypes.data  # noqa: E731
    # integer tables the port understands: label CSR over ALL keys of the
    # pods and working terms keyed by the same ids
    nk = cl.vals.shape[0]
    present = cl.vals >= 0
    cnt = present.sum(axis=0)
    lab_off = np.zeros(n + 1, np.int64)
    np.cumsum(cnt, out=lab_off[1:])
    order = np.argsort(~present.T, axis=1, kind="stable")  # keys of each pod first
    lab_key = np.concatenate([order[i, :cnt[i]] for i in range(n)]).astype(np.int32)
    lab_val = (cl.vals[lab_key, np.repeat(np.arange(n), cnt)].astype(np.int64)
               + lab_key.astype(np.int64) * 10_000_000)
    (so, sk, sv), (ao, ak, av) = cl.working_terms()
    sv2 = sv.astype(np.int64) + sk.astype(np.int64) * 10_000_000
    av2 = av.astype(np.int64) + ak.astype(np.int64) * 10_000_000
    allv = np.unique(np.concatenate([lab_val, sv2, av2]))
    lab_val = np.searchsorted(allv, lab_val).astype(np.int32)
    sv2 = np.searchsorted(allv, sv2).astype(np.int32)
    av2 = np.searchsorted(allv, av2).astype(np.int32)
    so = np.ascontiguousarray(so, np.int64)
    ao = np.ascontiguousarray(ao, np.int64)
    sk = np.ascontiguousarray(sk, np.int32)
    ak = np.ascontiguousarray(ak, np.int32)
    W = (n + 63) // 64
    threads = L.cpu_threads(0)
    M = np.empty(n * W, np.uint64)
    sel = np.empty(P * W, np.uint64)
    alw = np.empty(P * W, np.uint64)
    sec = {}
    t = time.perf_counter()
    L.cpu_build(n, nk, p(lab_off), p(lab_key), p(lab_val), P, p(so), p(sk), p(sv2), p(ao), p(ak),
                p(av2), p(M), p(sel), p(alw))
    sec["build_matrix"] = time.perf_counter() - t
    reach = np.empty(n, np.uint8)
    isol = np.empty(n, np.uint8)
    t = time.perf_counter()
    L.cpu_col_reduce(n, p(M), 0, p(reach))
    sec["all_reachable"] = time.perf_counter() - t
    t = time.perf_counter()
    L.cpu_col_reduce(n, p(M), 1, p(isol))
    sec["all_isolated"] = time.perf_counter() - t
    cross = np.empty(n, np.uint8)
    g = np.ascontiguousarray(gid, np.int32)
    t = time.perf_counter()
    L.cpu_crosscheck(n, p(M), p(g), p(cross))
    sec["user_crosscheck"] = time.perf_counter() - t
    t = time.perf_counter()
    row0 = np.unpackbits(M[:W].view(np.uint8), bitorder="little")[:n]
    sysiso = np.flatnonzero(row0 == 0).astype(np.int32)
    sec["system_isolation"] = time.perf_counter() - t
    t = time.perf_counter()
    off = np.zeros(n + 1, np.int64)
    L.cpu_lists(n, P, p(sel), p(off), None)
    lst = np.empty(max(1, int(off[-1])), np.int32)
    L.cpu_lists(n, P, p(sel), p(off), p(lst))
    cnt_pairs = ctypes.c_int64()
    cap = 1 << 24
    pairs = np.empty(2 * cap, np.int32)
    L.cpu_shadow(n, n, p(off), p(lst), p(alw), cap, p(pairs), ctypes.byref(cnt_pairs))
    sec["policy_shadow"] = time.perf_counter() - t
    total = sum(sec.values())
    res = {"all_reachable": np.flatnonzero(reach).astype(np.int32),
           "all_isolated": np.flatnonzero(isol).astype(np.int32),
           "user_crosscheck": np.flatnonzero(cross).astype(np.int32),
           "system_isolation": sysiso,
           "policy_shadow": pairs[:2 * min(cnt_pairs.value, cap)].reshape(-1, 2),
           "policy_shadow_count": cnt_pairs.value}
    verified, _ = verify_against_golden(config, cl, res, 1, 0, 0, "pairs")
    del M, sel, alw
    return {
        "value": float(n) * n / total, "unit": "pod-pairs/s", "cores": int(threads),
        "kind": "port",
        "sample": (f"the whole {n}-pod / {P}-policy cluster (no extrapolation): oracle/kano_cpu.c, "
                   f"kano_py's algorithm (build_matrix, all_reachable, all_isolated, "
                   f"user_crosscheck, system_isolation, policy_shadow) on {threads} OpenMP threads "
                   f"(OMP_NUM_THREADS); {total:.1f} s"),
        "seconds": {k: round(v, 3) for k, v in sec.items()},
        "verified": verified,
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --gpus N > 1 without torch.distributed.run: one process over N devices
    # (kano_group, SURVEY.md §8(b) kano_init(ngpu)): KANO_DEVICES (comma-
    # separated) or devices 0..N-1
    group = world == 1 and args.gpus > 1
    import torch
    dist = None
    if world > 1 or (args.shard_path and "RANK" in os.environ):
        import torch.distributed as dist
        # one GPU per rank; KANO_DIST_BACKEND=gloo with fewer GPUs than ranks
        # rehearses the N > 1 code path on one device (timings meaningless)
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group(os.environ.get("KANO_DIST_BACKEND", "nccl"))
    from kano import _native
    from kano._engine import DeviceBuild
    from kano._intern import tables_from_cluster
    from kano.synth import make_config, KEY_NAMES

    shadow = "off" if args.no_shadow else args.shadow
    if shadow == "auto":
        shadow = "count" if args.config in ("C4", "D1") else "pairs"
    cl = make_config(args.config)
    tables = tables_from_cluster(cl)
    n = cl.n
    gid = np.unique(cl.vals[KEY_NAMES.index("tenant")], return_inverse=True)[1].astype(np.int32)
    if group:
        return group_main(args, torch, cl, tables, gid, shadow)
    from kano.shard import row_range
    r0, r1 = row_range(n, world, rank)
    if args.rank_of > 1:
        r0, r1 = 0, n // args.rank_of
    # The engine runs on its own (high-priority) streams: the N > 1 exchange
    # is issued by the engine itself (native RCCL, or the emulated gather of
    # --rank-of), so no torch stream needs to order it.  (A torch stream
    # added a fifth queue beside the engine's four; GPU_MAX_HW_QUEUES is 4,
    # and streams sharing a hardware queue time-sliced the rank's kernels:
    # rank 0 of 8 took 0.61 ms a step instead of 0.46.)
    stream = None
    eng = DeviceBuild(None, device=torch.cuda.current_device(), path=args.path,
                      stream=stream.cuda_stream if stream is not None else None)
    # host -> device upload of the resident inputs (label tables, policy
    # terms, the tenant groups): reported apart from the step
    torch.cuda.synchronize()
    t_up = time.perf_counter()
    eng.upload(tables)
    eng.set_rows(r0, r1)
    up_tables_ms = (time.perf_counter() - t_up) * 1e3
    t_up = time.perf_counter()
    step = Step(eng, gid, n, rank, world, r0, r1, shadow=shadow, dist=dist,
                torch=torch, stream=stream, emulate=args.rank_of if args.rank_of > 1 else 0)
    up_groups_ms = (time.perf_counter() - t_up) * 1e3
    step.gather1 = bool(args.gather1) and not step.shard_path

    # (pipelined steps: the engine calls alone order its streams -- the fused
    # kano_verify, the emulated gather, the native RCCL gather; a torch
    # collective between the halves synchronises the device, so not there)
    pipelined = bool(args.pipeline) and (not step.shard_path or step.xchg.comm is not None
                                         or (step.xchg.dist is None and step.xchg.emulate_native))
    eng.set_pipeline(pipelined)

    def barrier():
        # (a queued prologue first: its gate would hold a device-wide sync;
        # the last timed step's queued prologue runs here, inside the timed
        # region -- one prologue more than the K steps need)
        eng.settle()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    # the pipelined calls' gates: how long each held the engine stream (its
    # idle time at the step boundary, device wall clock, no profiler)
    eng.gate_timing(reset=True)
    # k_rows' HIP-event times accumulate in the engine over the timed steps
    # (read once afterwards: kano_verify returns before its matrix write ends)
    eng.rows_timing(reset=True)
    eng.host_times(reset=True)
    eng.mfma_timing(reset=True)
    step.verify_max_ms = 0.0
    # Python's cyclic GC off in the timed region (as timeit does): a full
    # collection over torch's objects took ~7 ms between two steps
    import gc
    gc.collect()
    gc.disable()
    barrier()
    t0 = time.perf_counter()
    marks = []
    for _ in range(args.steps):
        step()
        marks.append(time.perf_counter())   # each step ends when its results are on the host
    barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    step_ms = np.diff(np.array([t0] + marks)) * 1e3
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    info = eng.info()
    ms_step = elapsed / args.steps * 1e3
    value = float(n) * n / (elapsed / args.steps)
    rt = eng.rows_timing()
    k_rows_ms = rt["sum_ms"] / rt["launches"] if rt["launches"] else float("nan")
    rows_kernel = {2: "k_rows", 3: "k_rows_w (k_rows_prep before it)",
                   4: "k_heavy_rows_t (every class heavy; k_ptrans before it, no k_rows)",
                   5: "k_heavy_rows_t then k_rows (timed from k_ptrans' start to k_rows' end)",
                   6: "k_heavy_rows_t then k_rows_w (timed from k_ptrans' start to k_rows_w's end)",
                   }.get(info["ROWS_KERNEL"], "none")
    mt = eng.mfma_timing()
    host = eng.host_times()
    gate = eng.gate_timing() if pipelined else None
    # k_rows alone (untimed, after the timed region): the same matrix write of
    # the same inputs with nothing beside it -- kano_build, which waits for its
    # write, so the write takes every CU (in the timed steps it runs on a
    # CU-masked stream beside the next step's build)
    eng.rows_timing(reset=True)
    eng.mfma_timing(reset=True)
    for _ in range(args.alone):
        eng.build()
    ra = eng.rows_timing()
    mta = eng.mfma_timing()
    alone_ms = ra["sum_ms"] / ra["launches"] if ra["launches"] else float("nan")
    rows_local = r1 - r0
    W = (n + 63) // 64
    alg_bytes = 8.0 * rows_local * W
    achieved = alg_bytes / (k_rows_ms * 1e-3) / 1e9 if k_rows_ms > 0 else 0.0
    res = step.results
    shadow_cnt = int(res.get("policy_shadow_count", -1))
    if dist is not None:
        t = torch.tensor([max(shadow_cnt, 0)], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        shadow_cnt = int(t.item())
    out = None
    traffic, traffic_src = (pmc_traffic(args.config, args.rank_of, info["ROWS_KERNEL"])
                            if world == 1 else (None, None))
    # the last step's results against kano_py's own outputs on this cluster
    # (tests/golden/expected/<config>.json); on row shards rank 0 checks the
    # combined column lists and the system row it owns
    if args.rank_of > 1:
        verified, vdetail = verify_shard_alone(args.config, cl, tables, gid, eng, step.results,
                                               r0, r1, shadow)
    else:
        verified, vdetail = verify_against_golden(args.config, cl, step.results, world, rank,
                                                 args.rank_of, shadow)
    if dist is not None:
        t = torch.tensor([0 if verified is False else 1], dtype=torch.int32, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if int(t.item()) == 0 and verified is not False:
            verified, vdetail = False, "another rank's results differ from the golden"
    box_fill = box_store_rate(torch, eng.W * 8 * max(r1 - r0, 1)) if world == 1 else None
    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "pod-pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u64", "data": "synthetic",
            "config": {"workload": WORKLOADS[args.config], "name": args.config, "pods": n,
                       "policies": cl.P, "mode": cl.mode, "seed": cl.seed,
                       "pipelined": pipelined,
                       "parallelism": (f"rows{world}" if args.rank_of <= 1 else
                                       f"rank 0 of {args.rank_of} emulated on one GPU, "
                                       "no collective (diagnostic, not a bench line)"),
                       "path": args.path,
                       "exchange": (step.xchg.mode if step.shard_path else "none (one rank, "
                                    "fused kano_verify)"),
                       "checks": "all_reachable, all_isolated, user_crosscheck(tenant), "
                                 "system_isolation(0)" +
                                 {"pairs": ", policy_shadow (pairs to the host)",
                                  "count": ", policy_shadow (every subset test; pair count "
                                           "only)",
                                  "off": ""}[shadow]},
            "verified": verified, "verified_against": vdetail,
            "upload_ms": {"tables": round(up_tables_ms, 3), "groups": round(up_groups_ms, 3),
                          "note": "host -> device input upload, once, outside the step"},
            "roofline": {"bound": "hbm", "kernel": rows_kernel, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "alg_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": k_rows_ms,
                         "launches_timed": rt["launches"],
                         "min_launch_ms": rt["min_ms"], "max_launch_ms": rt["max_ms"],
                         "box_fill_gbs": box_fill,
                         # the write runs beside the next step's build on a
                         # CU-masked stream when it is short enough to overlap
                         # it ("Pipelined steps")
                         "cus": info["ROWS_CUS"],
                         # the same launch alone on the device, every CU (a
                         # separate untimed measurement, see above)
                         "alone": ({"avg_launch_ms": alone_ms,
                                    "achieved": alg_bytes / (alone_ms * 1e-3) / 1e9,
                                    "frac": alg_bytes / (alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    "launches": ra["launches"],
                                    "how": "kano_build x %d after the timed region" % args.alone}
                                   if ra["launches"] else None)},
            # the dense path's MFMA contraction (k_heavy_gemm_f4 / k_heavy_mc_mfma,
            # block-scaled fp4 on 0/1 operands; --path mfma or AUTO's dense
            # choice): algorithmic ops / its event time, against the fp4
            # instruction's dense peak (and, for comparison with the round-5
            # int8 form, the int8 peak)
            "mfma_roofline": ({"bound": "mfma",
                               "kernel": {1: "k_heavy_mc_or (bitwise, timed for comparison)",
                                          2: "k_heavy_mc_mfma (split K, fp4)",
                                          3: "k_heavy_gemm_f4"}.get(info["HEAVY_KERNEL"], "none"),
                               "dtype": "fp4 e2m1 (0/1 operands), f32 accumulate",
                               "achieved": mt["ops_sum"] / (mt["sum_ms"] * 1e-3) / 1e12,
                               "peak": MFMA_F4_PEAK_TOPS, "unit": "TOP/s",
                               "frac": mt["ops_sum"] / (mt["sum_ms"] * 1e-3) / 1e12 /
                                       MFMA_F4_PEAK_TOPS,
                               "frac_vs_int8_peak": mt["ops_sum"] / (mt["sum_ms"] * 1e-3) / 1e12 /
                                                    MFMA_I8_PEAK_TOPS,
                               "ops_per_build": mt["ops_last"],
                               "avg_ms": mt["sum_ms"] / mt["builds"], "builds_timed": mt["builds"],
                               "heavy_classes": info["HEAVY"], "column_classes": info["UA"],
                               "policies": cl.P,
                               # in the timed steps the contraction shares the
                               # chip with the previous step's matrix write and
                               # this step's policy_shadow work; alone = the
                               # same launch in kano_build after the timed region
                               "alone": ({"avg_ms": mta["sum_ms"] / mta["builds"],
                                          "achieved": mta["ops_sum"] / (mta["sum_ms"] * 1e-3) / 1e12,
                                          "frac": mta["ops_sum"] / (mta["sum_ms"] * 1e-3) / 1e12 /
                                                  MFMA_F4_PEAK_TOPS,
                                          "frac_vs_int8_peak": mta["ops_sum"] /
                                                               (mta["sum_ms"] * 1e-3) / 1e12 /
                                                               MFMA_I8_PEAK_TOPS,
                                          "builds": mta["builds"]}
                                         if mta["builds"] and mta["sum_ms"] > 0 else None)}
                              if mt["builds"] > 0 and mt["sum_ms"] > 0 else None),
            "step_ms": {"min": round(float(step_ms.min()), 4),
                        "median": round(float(np.median(step_ms)), 4),
                        "p90": round(float(np.percentile(step_ms, 90)), 4),
                        "max": round(float(step_ms.max()), 4),
                        "worst5": [round(float(v), 3) for v in np.sort(step_ms)[-5:]],
                        "worst5_at": [int(i) for i in np.argsort(step_ms)[-5:]],
                        "engine_call_max": round(step.verify_max_ms, 4)},
            # kano_verify's host time by phase over the timed steps (us): a
            # stall names its phase (front = build + checks up to the column
            # words, back = lists + matrix-write launch + wait for the host
            # results, waits = the overlapped size syncs)
            "host_us": ({k: round(v, 1) for k, v in host.items() if k.endswith("_max")} |
                        {"front_mean": round(host["front_sum"] / max(1.0, host["calls"]), 1),
                         "back_mean": round(host["back_sum"] / max(1.0, host["calls"]), 1),
                         # the host's own time per call: the calls minus their
                         # waits for the device (size signals, the tail)
                         "waits_mean": round(host["wait_sum"] / max(1.0, host["calls"]), 1),
                         "tailwait_mean": round(host["tailwait_sum"] / max(1.0, host["calls"]), 1),
                         "issue_mean": round((host["front_sum"] + host["back_sum"] - host["wait_sum"]
                                              - host["tailwait_sum"]) / max(1.0, host["calls"]), 1),
                         "between_mean": round(host["gap_sum"] / max(1.0, host["calls"] - 1), 1)}
                        if host["calls"] > 0 else None),
            # the engine stream's idle time at the step boundary: how long each
            # pipelined call's gate held it (from the previous call's last
            # engine-stream kernel to this call's bell; device wall clock over
            # the last <= 64 timed steps, kano_gate_timing)
            "boundary_idle_us": ({"mean": round(gate["mean_us"], 1), "max": round(gate["max_us"], 1),
                                  "gates": gate["gates"]} if gate and gate["gates"] else None),
            "classes": info["U"], "nnz_select": info["NNZ_SEL"], "nnz_allow": info["NNZ_ALW"],
            "heavy_classes": info["HEAVY"], "shadow_pairs": shadow_cnt,
            "result_sizes": {k: int(len(v)) for k, v in res.items() if hasattr(v, "__len__")},
        }
        # (C2 / C3: kano_py's own policy_shadow list; C4's ~2.7e10 pairs fit no
        # host list, C5's matrix no host memory)
        if args.cold and world == 1 and args.rank_of <= 1 and n <= 200_000 and shadow == "pairs":
            out["cold_drop_in"] = cold_drop_in(cl, args.config)
        ref = kano_py_measured(args.config)
        if ref:
            out["kano_py_measured"] = ref
        if (args.cpu_baseline and world == 1 and args.rank_of <= 1 and n <= 200_000
                and shadow == "pairs"):
            out["cpu_baseline"] = cpu_baseline(cl, gid, args.config)
            out["cpu_baseline"]["cpu"] = _cpu_model()
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if verified is False:
        sys.exit(f"bench: results differ from the golden: {vdetail}")


class GroupStep:
    """The hot path over N devices in ONE process: kano_group_verify (every
    member's row shard built and checked at once on its own host thread, the
    members' column words exchanged -- ncclAllGather over xGMI between
    distinct devices, device copies between members sharing one -- and
    combined on every member; kano/multi.py MultiBuild)."""

    def __init__(self, eng, gid, n, shadow):
        from kano._engine import PinnedBuffer
        self.eng, self.n = eng, n
        self.shadow = shadow != "off"
        self.count_only = shadow == "count"
        eng.set_groups(gid)
        self.idx = np.empty(4 * max(n, 1), np.int32)
        self.pin = None
        self.pin_pairs = 0
        self.PinnedBuffer = PinnedBuffer
        self.results = {}
        self.verify_max_ms = 0.0

    def __call__(self):
        pairs = None
        if self.shadow and not self.count_only:
            if self.pin is None:
                self.pin_pairs = 1 << 20
                self.pin = self.PinnedBuffer(self.pin_pairs * 8)
                self.pairs_view = self.pin.view(np.int32, 2 * self.pin_pairs)
            pairs = self.pairs_view
        tv = time.perf_counter()
        r = self.eng.verify("stored", sys_row=0, shadow=self.shadow, pairs=pairs, idx=self.idx,
                            shadow_count_only=self.count_only)
        self.verify_max_ms = max(self.verify_max_ms, (time.perf_counter() - tv) * 1e3)
        res = {k: r[k] for k in ("all_reachable", "all_isolated", "user_crosscheck",
                                 "system_isolation") if r[k] is not None}
        if self.shadow:
            cnt = r["shadow_count"]
            res["policy_shadow"] = r["pairs"]
            res["policy_shadow_count"] = cnt
            if not self.count_only and cnt > self.pin_pairs:
                self.pin.close()
                self.pin_pairs = 2 * cnt
                self.pin = self.PinnedBuffer(self.pin_pairs * 8)
                self.pairs_view = self.pin.view(np.int32, 2 * self.pin_pairs)
        self.results = res
        return res


def group_main(args, torch, cl, tables, gid, shadow):
    """bench.py --gpus N (N > 1) without torch.distributed.run: the N row
    shards as members of one kano_group in this process; one JSON line."""
    from kano.multi import MultiBuild, requested_devices
    N = args.gpus
    devices = requested_devices(N) or list(range(N))
    n = cl.n
    t_up = time.perf_counter()
    eng = MultiBuild(tables, N, devices=devices, path=args.path, build=False)
    up_ms = (time.perf_counter() - t_up) * 1e3
    step = GroupStep(eng, gid, n, shadow)
    for _ in range(args.warmup):
        step()
    for m in eng.members:
        m.rows_timing(reset=True)
    # the exchange's own time: HIP events around it on member 0's stream
    eng.exchange_timing(enable=True, reset=True)
    import gc
    gc.collect()
    gc.disable()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for _ in range(args.steps):
        step()
        marks.append(time.perf_counter())
    for d in sorted(set(devices)):
        torch.cuda.synchronize(d)
    elapsed = time.perf_counter() - t0
    gc.enable()
    step_ms = np.diff(np.array([t0] + marks)) * 1e3
    W = (n + 63) // 64
    rows = []
    for m, (a, b) in zip(eng.members, eng.bounds):
        rt = m.rows_timing()
        ms = rt["sum_ms"] / rt["launches"] if rt["launches"] else float("nan")
        rows.append({"rows": [a, b], "avg_launch_ms": ms, "launches": rt["launches"],
                     "achieved": 8.0 * (b - a) * W / (ms * 1e-3) / 1e9 if ms > 0 else 0.0})
    xt = eng.exchange_timing(enable=False)
    # the dominant kernel's roofline: member 0's matrix write (its row shard);
    # every member's beside it
    r0 = rows[0]
    fr = [r["achieved"] / HBM_PEAK_GBS for r in rows]
    verified, vdetail = verify_against_golden(args.config, cl, step.results, 1, 0, 0, shadow)
    out = {
        "metric": METRIC, "value": float(n) * n / (elapsed / args.steps), "unit": "pod-pairs/s",
        "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": WORKLOADS[args.config], "name": args.config, "pods": n,
                   "policies": cl.P, "mode": cl.mode, "seed": cl.seed,
                   "parallelism": f"rows{N} in one process (kano_group, {eng.mode})",
                   "devices": devices, "path": args.path,
                   "exchange": eng.mode,
                   "exchange_mode": 1 if eng.mode.startswith("rccl") else 2,
                   "checks": "all_reachable, all_isolated, user_crosscheck(tenant), "
                             "system_isolation(0)" +
                             {"pairs": ", policy_shadow (pairs to the host)",
                              "count": ", policy_shadow (pair count only)", "off": ""}[shadow]},
        "verified": verified, "verified_against": vdetail,
        "upload_ms": {"group_create_and_tables": round(up_ms, 3)},
        "roofline": {"bound": "hbm", "kernel": "k_rows (member 0)", "achieved": r0["achieved"],
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": r0["achieved"] / HBM_PEAK_GBS, "traffic": None,
                     "alg_bytes_per_launch": 8.0 * (r0["rows"][1] - r0["rows"][0]) * W,
                     "avg_launch_ms": r0["avg_launch_ms"], "launches_timed": r0["launches"],
                     "members": rows, "member_frac_min": min(fr), "member_frac_max": max(fr)},
        "exchange_ms": {"what": f"{3 * W} u64 words per member ({eng.mode}), HIP events on "
                                "member 0's stream around the exchange",
                        "calls": xt["calls"], "avg": xt["avg_ms"], "max": xt["max_ms"]},
        "step_ms": {"min": round(float(step_ms.min()), 4),
                    "median": round(float(np.median(step_ms)), 4),
                    "p90": round(float(np.percentile(step_ms, 90)), 4),
                    "max": round(float(step_ms.max()), 4),
                    "engine_call_max": round(step.verify_max_ms, 4)},
        "result_sizes": {k: int(len(v)) for k, v in step.results.items()
                         if hasattr(v, "__len__")},
    }
    print(json.dumps(out), flush=True)
    eng.close()
    if verified is False:
        sys.exit(f"bench: results differ from the golden: {vdetail}")


def _golden(config):
    path = os.path.join(ROOT, "tests", "golden", "expected", f"{config}.json")
    try:
        with open(path) as f:
            return json.load(f), os.path.relpath(path, ROOT)
    except OSError:
        return None, None


def _list_ok(got, exp):
    import hashlib
    got = np.ascontiguousarray(np.asarray(got, dtype=np.int32))
    if isinstance(exp, dict):
        return (got.shape[0] == exp["count"] and
                hashlib.sha256(got.tobytes()).hexdigest() == exp["sha256"])
    return got.tolist() == exp


def verify_against_golden(config, cl, res, world, rank, rank_of, shadow):
    """True / False against the record of this exact cluster: kano_py's own
    (C2-C4, tests/golden/make_golden.py), or for C5, out of kano_py's reach,
    the indexed restatement's (tests/golden/make_c5.py, oracle/kano_indexed.py,
    pinned on C2-C4 against kano_py); None when there is no record or the run
    is an emulated diagnostic."""
    import hashlib
    exp, src = _golden(config)
    if exp is None:
        return None, "no record for this config"
    if rank_of > 1:
        return None, "emulated shard step (other ranks' words are zero): not checked"
    if exp.get("seed", {}).get("fingerprint") != cl.fingerprint():
        return False, f"{src}: cluster fingerprint differs"
    bad = []
    for k in ("all_reachable", "all_isolated"):
        if not _list_ok(res[k], exp[k]):
            bad.append(k)
    if not _list_ok(res["user_crosscheck"], exp["user_crosscheck"]["result"]):
        bad.append("user_crosscheck")
    if "system_isolation" in res and not _list_ok(res["system_isolation"],
                                                  exp["system_isolation"]["result"]):
        bad.append("system_isolation")
    sh = exp["policy_shadow"]
    if shadow == "pairs" and world == 1:
        if res["policy_shadow_count"] != sh["count"] or hashlib.sha256(
                np.ascontiguousarray(res["policy_shadow"], dtype=np.int32).tobytes()
        ).hexdigest() != sh["sha256"]:
            bad.append("policy_shadow")
    elif shadow != "off" and world == 1:
        want = sh.get("count", sh.get("oracle_count"))
        if res["policy_shadow_count"] != want:
            bad.append("policy_shadow count")
    if bad:
        return False, f"{src}: {', '.join(bad)} differ"
    what = "lists" + (", policy_shadow " + ("pairs sha256" if shadow == "pairs" else "count")
                      if shadow != "off" and world == 1 else "")
    who = exp.get("source", "kano_py on the same seeded cluster")
    return True, f"{src} ({who}): {what} equal"


def verify_shard_alone(config, cl, tables, gid, eng, res, r0, r1, shadow):
    """--rank-of N: what rank 0's shard can check without the other ranks'
    words (the emulated gather leaves them zero, so its column lists are
    partial).  After the timed region, one unsharded build of the same cluster
    is verified against the record (verify_against_golden); then the shard's
    rows must equal that build's rows [r0, r1) (per-row digests), its
    policy_shadow pairs the full list's first ones (pairs are emitted per pod
    in row order, algorithm.py:58-80, and rank 0 holds rows from 0), and its
    system_isolation(0) list the record's (row 0 is rank 0's)."""
    from kano._engine import DeviceBuild
    assert r0 == 0
    shard = {k: np.array(v, copy=True) for k, v in res.items()
             if v is not None and hasattr(v, "__len__")}
    cnt = int(res.get("policy_shadow_count", -1))
    full = DeviceBuild(tables, build=False)
    try:
        fr = full.verify(gid, sys_row=0, shadow=shadow != "off",
                         shadow_count_only=shadow == "count")
        fres = {k: fr[k] for k in ("all_reachable", "all_isolated", "user_crosscheck",
                                   "system_isolation")}
        if shadow != "off":
            fres["policy_shadow"] = fr["pairs"]
            fres["policy_shadow_count"] = fr["shadow_count"]
        ok, detail = verify_against_golden(config, cl, fres, 1, 0, 0, shadow)
        if ok is not True:
            return ok, "unsharded build: " + detail
        bad = []
        if not np.array_equal(eng.rows_digest(r0, r1 - r0), full.rows_digest(r0, r1 - r0)):
            bad.append("row digests")
        if not np.array_equal(np.asarray(shard.get("system_isolation", []), np.int32),
                              np.asarray(fres["system_isolation"], np.int32)):
            bad.append("system_isolation")
        if shadow == "pairs":
            fp = np.asarray(fres["policy_shadow"], np.int32).reshape(-1, 2)
            sp = np.asarray(shard["policy_shadow"], np.int32).reshape(-1, 2)
            if cnt > fp.shape[0] or not np.array_equal(sp[:cnt], fp[:cnt]):
                bad.append("policy_shadow pairs")
    finally:
        full.close()
    if bad:
        return False, f"rank 0 of the shards: {', '.join(bad)} differ from the unsharded build"
    what = "row digests, system_isolation" + (", policy_shadow pairs (prefix of the full list)"
                                              if shadow == "pairs" else "")
    return True, (f"rank 0's shard [{r0}, {r1}) against an unsharded build verified by "
                  f"{detail}: {what} equal (the column lists need every rank's words: not "
                  "checked here)")


def kano_py_measured(config):
    """kano_py's own times on this cluster, measured in the build container
    by tests/golden/make_golden.py (single thread, bitarray 2.3.0)."""
    exp, src = _golden(config)
    if exp is None or "reference_seconds" not in exp:
        return None
    t = exp["reference_seconds"]
    total = float(sum(t.values()))
    n = exp["n"]
    return {"seconds": {k: round(v, 2) for k, v in t.items()}, "total_s": round(total, 1),
            "pod_pairs_per_s": n * n / total, "cores": 1,
            "where": "build container (Intel Xeon, py3.9, bitarray 2.3.0), not the GPU box",
            "complete": "policy_shadow" in t, "source": src}


def box_store_rate(torch, nbytes):
    """This box's plain device fill rate on a buffer of the matrix's size
    (torch fill_, HIP events): context for the k_rows roofline fraction,
    boxes differ by up to 20 %."""
    try:
        buf = torch.empty(int(nbytes) // 8, dtype=torch.int64, device="cuda")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        buf.fill_(1)
        ms = []
        for _ in range(5):
            ev[0].record()
            buf.fill_(0)
            ev[1].record()
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        del buf
        return round(nbytes / (min(ms) * 1e-3) / 1e9, 1)
    except Exception:   # noqa: BLE001 (context only)
        return None


def pmc_traffic(config, rank_of=0, rows_kernel=2):
    """HBM bytes per launch of the matrix write's main kernel (k_rows, or
    k_rows_w for wide rows) from the committed PMC summary of this workload
    (scripts/pmc.sh: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this
    same bench command, FETCH doubled for gfx950): profiles/pmc_<config>.json,
    pmc_<config>r<N>.json for --rank-of N."""
    name = f"pmc_{config}" + (f"r{rank_of}" if rank_of > 1 else "") + ".json"
    path = os.path.join(ROOT, "profiles", name)
    want = "kano::k_rows_w<" if rows_kernel in (3, 6) else "kano::k_rows<"
    try:
        with open(path) as f:
            d = json.load(f)
        # the kernel's name as rocprofv3 prints it ("void kano::k_rows<256>")
        k = next(v for nm, v in d["kernels"].items() if want in nm)
        return float(k["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT)
    except (OSError, KeyError, ValueError, TypeError, StopIteration):
        return None, None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
