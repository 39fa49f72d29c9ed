"""One device-resident build of the reachability matrix (a kano_ctx).

Thin Python wrapper of the C ABI (include/kano_hip.h): uploads interned
tables, runs the build and the checks, and hands results back as numpy
arrays.  The drop-in API (model.py / algorithm.py) and the benchmark both
drive the engine through this class.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_int64, c_void_p
from typing import Optional, Tuple

import numpy as np

from . import _native as nat
from ._intern import Tables


def _ptr(a: Optional[np.ndarray]):
    # the address as an int: the argtypes are c_void_p, and ctypes converts
    # an int much faster than numpy's data_as builds a pointer object
    return None if a is None else a.ctypes.data


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) viewed as a numpy array; D2H
    copies into it run at the full PCIe rate."""

    def __init__(self, nbytes: int):
        self._lib = nat.load()
        self._p = c_void_p()
        self.nbytes = max(int(nbytes), 16)
        nat.check(None, self._lib.kano_host_alloc(self.nbytes, byref(self._p)), "kano_host_alloc")

    def view(self, dtype, count: int) -> np.ndarray:
        dt = np.dtype(dtype)
        if count * dt.itemsize > self.nbytes:
            raise ValueError("pinned buffer too small")
        buf = (ctypes.c_char * (count * dt.itemsize)).from_address(self._p.value)
        return np.frombuffer(buf, dtype=dt, count=count)

    def close(self):
        if self._p:
            self._lib.kano_host_free(self._p)
            self._p = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuild:
    """A kano_ctx holding one build (or one row shard of it) on one GPU."""

    def __init__(self, tables: Optional[Tables] = None, device: int = 0,
                 rows: Optional[Tuple[int, int]] = None, path: str = "auto",
                 stream: Optional[int] = None, build: bool = True, lean: bool = False):
        self.lib = nat.load()
        self.ctx = c_void_p()
        self._owned = True            # close() destroys the context (not when adopted)
        # lean: kano_create_lean (no CU-masked write stream: builds the caller
        # waits for, the drop-in build_matrix)
        create = self.lib.kano_create_lean if lean else self.lib.kano_create
        rc = create(int(device), byref(self.ctx))
        if rc != 0:
            self.ctx = c_void_p()
            raise nat.KanoNativeError(
                f"kano_create(device={device}) failed (rc={rc}): no usable HIP device")
        self.device = device
        self.path = path
        self._counts = None
        self.row_span = None          # (r0, r1) when this context holds a row shard
        if stream is not None:
            self._chk(self.lib.kano_set_stream(self.ctx, c_void_p(stream)), "kano_set_stream")
        self.tables = None
        if tables is not None:
            self.upload(tables)
            if rows is not None:
                self.set_rows(*rows)
            if build:
                self.build(path)

    @classmethod
    def adopt(cls, ctx: c_void_p, device: int = 0, path: str = "auto") -> "DeviceBuild":
        """Wrap a context owned elsewhere (a kano_group member, kano/multi.py):
        its owner destroys it: this wrapper never does (close() only drops
        the handle)."""
        self = cls.__new__(cls)
        self.lib = nat.load()
        self.ctx = ctx
        self._owned = False
        self.device = device
        self.path = path
        self._counts = None
        self.row_span = None
        self.tables = None
        return self

    # -- plumbing -------------------------------------------------------
    def _chk(self, rc, what):
        nat.check(self.ctx, rc, what)

    def close(self):
        if self.ctx:
            if getattr(self, "_owned", True):
                self.lib.kano_destroy(self.ctx)
            self.ctx = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- inputs / build -------------------------------------------------
    def upload(self, t: Tables) -> None:
        self.tables = t
        self.row_span = None          # kano_set_pods resets the engine to every row
        pv = np.ascontiguousarray(t.pod_val, dtype=np.int32)
        self._chk(self.lib.kano_set_pods(self.ctx, t.n, t.ncols, _ptr(pv)), "kano_set_pods")
        if getattr(t, "expr_col", None) is not None and len(t.expr_col):
            ex = [np.ascontiguousarray(a, dtype=d) for a, d in (
                (t.expr_col, np.int32), (t.expr_op, np.int32), (t.expr_off, np.int64),
                (t.expr_val, np.int32))]
            self._chk(self.lib.kano_set_expressions(self.ctx, len(ex[0]), *[_ptr(a) for a in ex]),
                      "kano_set_expressions")
        arrs = [np.ascontiguousarray(a, dtype=d) for a, d in (
            (t.sel_off, np.int64), (t.sel_col, np.int32), (t.sel_val, np.int32),
            (t.alw_off, np.int64), (t.alw_col, np.int32), (t.alw_val, np.int32))]
        self._chk(self.lib.kano_set_policies(self.ctx, t.P, *[_ptr(a) for a in arrs]),
                  "kano_set_policies")

    def set_rows(self, r0: int, r1: int) -> None:
        self._chk(self.lib.kano_set_shard(self.ctx, int(r0), int(r1)), "kano_set_shard")
        n = self.info()["N"]          # the engine's own pod count (tables may be absent)
        self.row_span = None if (int(r0), int(r1)) == (0, n) else (int(r0), int(r1))

    @property
    def is_shard(self) -> bool:
        return self.row_span is not None

    def build(self, path: Optional[str] = None) -> None:
        p = nat.PATHS[path or self.path]
        self._chk(self.lib.kano_build(self.ctx, p), "kano_build")

    def build_classes(self, path: Optional[str] = None) -> None:
        """kano_build_classes: the build up to the class-level matrix; M is
        written on first use."""
        p = nat.PATHS[path or self.path]
        self._chk(self.lib.kano_build_classes(self.ctx, p), "kano_build_classes")

    def info(self) -> dict:
        out = np.zeros(nat.INFO_SLOTS, dtype=np.int64)
        self._chk(self.lib.kano_info(self.ctx, _ptr(out)), "kano_info")
        return {k: int(out[v]) for k, v in nat.INFO.items()}

    @property
    def n(self) -> int:
        return self.tables.n

    @property
    def W(self) -> int:
        return (self.tables.n + 63) >> 6

    @staticmethod
    def empty(n: int, device: int = 0, rows: Optional[Tuple[int, int]] = None) -> "DeviceBuild":
        """A context holding an n x n matrix (or its rows [r0, r1)) and no
        policies (the target of put_rows or of path_from / path_combine)."""
        z64 = np.zeros(1, np.int64)
        e = np.zeros(0, np.int32)
        t = Tables(int(n), 0, np.zeros((0, int(n)), np.int32), z64, e, e, z64, e, e)
        return DeviceBuild(t, device=device, rows=rows)

    def path_from(self, src: "DeviceBuild", hops: int = 2, mode: str = "auto") -> dict:
        """This context's matrix := the multi-hop reachability of src's
        matrix (kano_path; kubesv/kubesv/constraint.py:233-237)."""
        info = np.zeros(6, dtype=np.int64)
        self._chk(self.lib.kano_path(src.ctx, self.ctx, int(hops), nat.PATHS[mode], _ptr(info)),
                  "kano_path")
        keys = ("steps", "steps_run", "mfma_steps", "row_classes", "col_classes", "identity")
        return {k: int(v) for k, v in zip(keys, info)}

    def export_rows(self, r0: int, nrows: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Rows as bitarray bytes (big-endian bit order), (nrows, ceil(n/8))."""
        nb = (self.tables.n + 7) >> 3
        if out is None:
            out = np.empty((max(nrows, 0), nb), dtype=np.uint8)
        self._chk(self.lib.kano_export_rows(self.ctx, int(r0), int(nrows), _ptr(out)),
                  "kano_export_rows")
        return out

    def import_rows(self, r0: int, rows: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.uint8)
        self._chk(self.lib.kano_import_rows(self.ctx, int(r0), int(rows.shape[0]), _ptr(rows)),
                  "kano_import_rows")

    def k8s_edge_from(self, in_t: "DeviceBuild", eg_t: "DeviceBuild", self_traffic: bool,
                      all_pairs: bool, pods: bool = False, dst_is_egress: bool = False) -> int:
        """This context's matrix := kubesv's edge relation from the two
        per-direction builds (kano_k8s_edge; kubesv/kubesv/constraint.py:191-231).
        Returns the bits the product added beyond the self term."""
        info = np.zeros(1, dtype=np.int64)
        flags = ((1 if self_traffic else 0) | (2 if all_pairs else 0) | (4 if pods else 0) |
                 (8 if dst_is_egress else 0))
        self._chk(self.lib.kano_k8s_edge(in_t.ctx, eg_t.ctx, self.ctx, flags, _ptr(info)),
                  "kano_k8s_edge")
        return int(info[0])

    def path_shard_words(self) -> int:
        w = c_int64(0)
        self._chk(self.lib.kano_path_shard_words(self.ctx, byref(w)), "kano_path_shard_words")
        return int(w.value)

    def path_shard(self, t_dev_ptr: int) -> None:
        """This row shard's part of the path's one-hop table (device memory)."""
        self._chk(self.lib.kano_path_shard(self.ctx, c_void_p(t_dev_ptr)), "kano_path_shard")

    def path_combine(self, src: "DeviceBuild", gathered_dev_ptr: int, nranks: int,
                     hops: int = 2, mode: str = "auto") -> dict:
        """This context's rows := src's shard of the path matrix, from the
        ranks' gathered parts."""
        info = np.zeros(6, dtype=np.int64)
        self._chk(self.lib.kano_path_combine(src.ctx, self.ctx, c_void_p(gathered_dev_ptr),
                                             int(nranks), int(hops), nat.PATHS[mode],
                                             _ptr(info)), "kano_path_combine")
        keys = ("steps", "steps_run", "mfma_steps", "row_classes", "col_classes", "identity")
        return {k: int(v) for k, v in zip(keys, info)}

    # -- incremental updates ---------------------
    def add_policies(self, xval: np.ndarray, sel_csr, alw_csr) -> int:
        """Append policies (terms in this build's id space, kano._intern.
        intern_more); returns the first new engine id."""
        so, sc, sv = (np.ascontiguousarray(a, dtype=d) for a, d in
                      zip(sel_csr, (np.int64, np.int32, np.int32)))
        ao, ac, av = (np.ascontiguousarray(a, dtype=d) for a, d in
                      zip(alw_csr, (np.int64, np.int32, np.int32)))
        xv = np.ascontiguousarray(xval, dtype=np.int32)
        first = c_int64(0)
        self._chk(self.lib.kano_add_policies(
            self.ctx, int(so.shape[0] - 1), int(xv.shape[0]), _ptr(xv), _ptr(so), _ptr(sc),
            _ptr(sv), _ptr(ao), _ptr(ac), _ptr(av), byref(first)), "kano_add_policies")
        return int(first.value)

    def remove_policies(self, ids) -> None:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.int64).reshape(-1))
        self._chk(self.lib.kano_remove_policies(self.ctx, int(a.shape[0]), _ptr(a)),
                  "kano_remove_policies")

    def added_policy_sets(self, eid: int) -> Tuple[np.ndarray, np.ndarray]:
        W = self.W
        s = np.zeros(W, dtype=np.uint64)
        a = np.zeros(W, dtype=np.uint64)
        self._chk(self.lib.kano_added_policy_sets(self.ctx, int(eid), _ptr(s), _ptr(a)),
                  "kano_added_policy_sets")
        return s, a

    # -- checks ---------------------------------------------------------
    def col_checks(self) -> Tuple[np.ndarray, np.ndarray]:
        W = self.W
        ca = np.zeros(W, dtype=np.uint64)
        co = np.zeros(W, dtype=np.uint64)
        self._chk(self.lib.kano_col_checks(self.ctx, _ptr(ca), _ptr(co)), "kano_col_checks")
        return ca, co

    def crosscheck(self, gid: np.ndarray) -> np.ndarray:
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        if gid.shape[0] != self.n:
            raise ValueError("gid must have one entry per pod")
        out = np.zeros(self.W, dtype=np.uint64)
        self._chk(self.lib.kano_crosscheck(self.ctx, _ptr(gid), _ptr(out)), "kano_crosscheck")
        return out

    def col_flags_dev(self, flags_dev_ptr: int) -> None:
        self._chk(self.lib.kano_col_flags_dev(self.ctx, c_void_p(flags_dev_ptr)),
                  "kano_col_flags_dev")

    def crosscheck_dev(self, gid: np.ndarray, flags_dev_ptr: int) -> None:
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        self._chk(self.lib.kano_crosscheck_dev(self.ctx, _ptr(gid), c_void_p(flags_dev_ptr)),
                  "kano_crosscheck_dev")

    # -- matrix access --------------------------------------------------
    def rows(self, r0: int, nrows: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        if out is None:
            out = np.zeros((nrows, self.W), dtype=np.uint64)
        self._chk(self.lib.kano_get_rows(self.ctx, int(r0), int(nrows), _ptr(out)),
                  "kano_get_rows")
        return out

    def rows_digest(self, r0: int, nrows: int) -> np.ndarray:
        """kano_rows_digest: one 64-bit digest per row (tests/_golden.py
        row_digest computes the same on the host)."""
        out = np.zeros(max(nrows, 1), dtype=np.uint64)
        self._chk(self.lib.kano_rows_digest(self.ctx, int(r0), int(nrows), _ptr(out)),
                  "kano_rows_digest")
        return out[:nrows]

    def put_rows(self, r0: int, words: np.ndarray) -> None:
        words = np.ascontiguousarray(words, dtype=np.uint64).reshape(-1, self.W)
        self._chk(self.lib.kano_put_rows(self.ctx, int(r0), words.shape[0], _ptr(words)),
                  "kano_put_rows")

    def col(self, j: int) -> np.ndarray:
        info = self.info()
        rl = info["ROW1"] - info["ROW0"]
        out = np.zeros((rl + 63) >> 6, dtype=np.uint64)
        self._chk(self.lib.kano_get_col(self.ctx, int(j), _ptr(out)), "kano_get_col")
        return out

    def get_bit(self, i: int, j: int) -> int:
        v = c_int()
        self._chk(self.lib.kano_get_bit(self.ctx, int(i), int(j), byref(v)), "kano_get_bit")
        return int(v.value)

    def set_bit(self, i: int, j: int, value) -> None:
        self._chk(self.lib.kano_set_bit(self.ctx, int(i), int(j), 1 if value else 0),
                  "kano_set_bit")

    def policy_sets(self, p: int, sel: bool = True, allow: bool = True):
        if self.tables is not None and p >= self.tables.P:   # an added policy
            s, a = self.added_policy_sets(p)
            return (s if sel else None), (a if allow else None)
        W = self.W
        s = np.zeros(W, dtype=np.uint64) if sel else None
        a = np.zeros(W, dtype=np.uint64) if allow else None
        self._chk(self.lib.kano_get_policy_sets(self.ctx, int(p), _ptr(s), _ptr(a)),
                  "kano_get_policy_sets")
        return s, a

    def classes(self) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.int32)
        self._chk(self.lib.kano_get_classes(self.ctx, _ptr(out)), "kano_get_classes")
        return out

    def select_csr(self) -> Tuple[np.ndarray, np.ndarray]:
        info = self.info()
        off = np.zeros(info["U"] + 1, dtype=np.int64)
        pol = np.zeros(max(info["NNZ_SEL"], 1), dtype=np.int32)
        self._chk(self.lib.kano_get_select_csr(self.ctx, _ptr(off), _ptr(pol)),
                  "kano_get_select_csr")
        return off, pol[: info["NNZ_SEL"]]

    def allow_csr(self) -> Tuple[np.ndarray, np.ndarray]:
        info = self.info()
        off = np.zeros(info["P"] + 1, dtype=np.int64)
        pods = np.zeros(max(info["NNZ_ALW"], 1), dtype=np.int32)
        self._chk(self.lib.kano_get_allow_csr(self.ctx, _ptr(off), _ptr(pods)),
                  "kano_get_allow_csr")
        return off, pods[: info["NNZ_ALW"]]

    # -- policy checks --------------------------------------------------
    def shadow_count(self) -> int:
        cnt = c_int64()
        self._chk(self.lib.kano_shadow(self.ctx, byref(cnt)), "kano_shadow")
        return int(cnt.value)

    def shadow_fetch(self, count: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        if out is None:
            out = np.zeros((count, 2), dtype=np.int32)
        self._chk(self.lib.kano_shadow_fetch(self.ctx, _ptr(out)), "kano_shadow_fetch")
        return out

    def shadow(self) -> np.ndarray:
        return self.shadow_fetch(self.shadow_count())

    def set_groups(self, gid: np.ndarray, ngroups: int = 0) -> None:
        """kano_set_groups: upload the pods' group ids once (resident input);
        then ``verify(gid="stored")`` runs user_crosscheck on them."""
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        if gid.shape[0] != self.n:
            raise ValueError("gid must have one entry per pod")
        self._chk(self.lib.kano_set_groups(self.ctx, _ptr(gid), int(ngroups)), "kano_set_groups")

    def _result_slots(self) -> None:
        # reused result slots (no per-call allocation)
        self._counts = np.zeros(4, dtype=np.int64)
        self._counts_p = self._counts.ctypes.data
        self._cnt = c_int64(0)
        self._cnt_ref = byref(self._cnt)
        self._bufs = (None, None, None, None)

    def _buf_ptrs(self, idx, pairs):
        # the caller's reused idx / pairs buffers: their addresses once (the
        # held references keep both arrays, and so their addresses, alive)
        b_idx, p_idx, b_pairs, p_pairs = self._bufs
        if idx is not b_idx or pairs is not b_pairs:
            b_idx, p_idx, b_pairs, p_pairs = idx, _ptr(idx), pairs, _ptr(pairs)
            self._bufs = (b_idx, p_idx, b_pairs, p_pairs)
        return p_idx, p_pairs

    def verify(self, gid=None, sys_row: int = 0, shadow: bool = True,
               pairs: Optional[np.ndarray] = None, idx: Optional[np.ndarray] = None,
               ngroups: int = 0, path: Optional[str] = None,
               shadow_count_only: bool = False) -> dict:
        """kano_verify: build + every check in one call (three host syncs).

        Returns the reference's result lists as int32 index arrays
        (``all_reachable``, ``all_isolated``, ``user_crosscheck`` (None without
        gid), ``system_isolation`` (None when sys_row is not in this shard))
        and, with ``shadow``, ``shadow_count`` plus ``pairs`` (a (count, 2)
        view of the given buffer when it is large enough, else fetched
        afterwards).  ``idx`` (>= 4*n int32, e.g. pinned) receives the lists.
        ``ngroups`` > 0 declares ``gid < ngroups`` (checked on the device).
        ``shadow_count_only``: policy_shadow's subset tests run and its pair
        count is returned, the pairs are not emitted (``pairs`` is None)."""
        n = self.n
        if idx is None:
            idx = np.empty(max(4 * n, 1), dtype=np.int32)
        elif idx.size < 4 * n:
            raise ValueError("idx buffer needs 4*n entries")
        stored = isinstance(gid, str) and gid == "stored"
        if stored:
            gid, ngroups = None, nat.STORED_GROUPS
        elif gid is not None:
            if not (isinstance(gid, np.ndarray) and gid.dtype == np.int32
                    and gid.flags.c_contiguous):
                gid = np.ascontiguousarray(gid, dtype=np.int32)
            if gid.shape[0] != n:
                raise ValueError("gid must have one entry per pod")
        if self._counts is None:
            self._result_slots()
        counts, cnt = self._counts, self._cnt
        cap = 0 if pairs is None else pairs.size // 2
        if shadow_count_only:
            cap = -1
        p_idx, p_pairs = self._buf_ptrs(idx, pairs)
        pth = nat.PATHS[path or self.path]
        rc = self.lib.kano_verify(self.ctx, pth, _ptr(gid), int(ngroups), int(sys_row), p_idx,
                                  self._counts_p, p_pairs, int(cap),
                                  self._cnt_ref if shadow else None)
        if rc != 0:
            self._chk(rc, "kano_verify")
        out, o = {}, 0
        for name, k in zip(("all_reachable", "all_isolated", "user_crosscheck",
                            "system_isolation"), counts.tolist()):
            out[name] = idx[o:o + k] if k >= 0 else None
            o += max(k, 0)
        if gid is None and not stored:
            out["user_crosscheck"] = None
        if shadow:
            k = int(cnt.value)
            out["shadow_count"] = k
            if shadow_count_only:
                out["pairs"] = None
            elif pairs is not None and k <= cap:
                out["pairs"] = pairs.reshape(-1)[:2 * k].reshape(k, 2)
            else:
                out["pairs"] = self.shadow_fetch(k)
        return out

    def verify_shard(self, words_dev_ptr: int, gid=None, sys_row: int = 0, shadow: bool = True,
                     ngroups: int = 0, path: Optional[str] = None,
                     shadow_count_only: bool = False) -> None:
        """kano_verify_shard: build this row shard and run its checks up to the
        column words, written (3*W u64, [OR | cross | NAND]) to the device
        buffer at ``words_dev_ptr``.  Asynchronous on the engine's stream;
        gather the ranks' words on that stream, then ``verify_combine``."""
        self._gid_keep = None
        if isinstance(gid, str) and gid == "stored":
            gid, ngroups = None, nat.STORED_GROUPS
        elif gid is not None:
            gid = np.ascontiguousarray(gid, dtype=np.int32)
            if gid.shape[0] != self.n:
                raise ValueError("gid must have one entry per pod")
            self._gid_keep = gid
        self._shard_shadow = bool(shadow)
        pth = nat.PATHS[path or self.path]
        mode = (2 if shadow_count_only else 1) if shadow else 0
        self._chk(self.lib.kano_verify_shard(self.ctx, pth, _ptr(gid), int(ngroups), int(sys_row),
                                             mode, c_void_p(words_dev_ptr)),
                  "kano_verify_shard")

    def verify_gather(self, comm_ptr: int, nranks: int, gid=None, sys_row: int = 0,
                      shadow: bool = True, pairs: Optional[np.ndarray] = None,
                      idx: Optional[np.ndarray] = None, ngroups: int = 0,
                      path: Optional[str] = None, shadow_count_only: bool = False) -> dict:
        """kano_verify_gather: ``verify_shard``, the ranks' all-gather and
        ``verify_combine`` in one engine call, the all-gather issued by the
        engine on its stream through the RCCL communicator ``comm_ptr``
        (an ncclComm_t over ``nranks`` ranks, e.g. torch's
        ``ProcessGroupNCCL._comm_ptr()``).  Results as ``verify_combine``."""
        if isinstance(gid, str) and gid == "stored":
            gid, ngroups = None, nat.STORED_GROUPS
        elif gid is not None:
            gid = np.ascontiguousarray(gid, dtype=np.int32)
            if gid.shape[0] != self.n:
                raise ValueError("gid must have one entry per pod")
        self._shard_shadow = bool(shadow)
        pth = nat.PATHS[path or self.path]
        mode = (2 if shadow_count_only else 1) if shadow else 0
        return self._combine_call(
            lambda idx_p, cnt_p, pairs_p, cap, cnt_ref: self.lib.kano_verify_gather(
                self.ctx, pth, _ptr(gid), int(ngroups), int(sys_row), mode, c_void_p(comm_ptr),
                int(nranks), idx_p, cnt_p, pairs_p, cap, cnt_ref),
            "kano_verify_gather", pairs, idx, shadow_count_only)

    def checks_shard(self, words_dev_ptr: int, gid=None, sys_row: int = 0,
                     ngroups: int = 0) -> None:
        """kano_checks_shard: this shard's column words from the matrix as
        it stands (after add_policies / remove_policies); finish with
        ``verify_combine``."""
        self._gid_keep = None
        if isinstance(gid, str) and gid == "stored":
            gid, ngroups = None, nat.STORED_GROUPS
        elif gid is not None:
            gid = np.ascontiguousarray(gid, dtype=np.int32)
            if gid.shape[0] != self.n:
                raise ValueError("gid must have one entry per pod")
            self._gid_keep = gid
        self._shard_shadow = False
        self._chk(self.lib.kano_checks_shard(self.ctx, _ptr(gid), int(ngroups), int(sys_row),
                                             c_void_p(words_dev_ptr)), "kano_checks_shard")

    def verify_combine(self, gathered_dev_ptr: int, nranks: int, cross: bool = True,
                       pairs: Optional[np.ndarray] = None,
                       idx: Optional[np.ndarray] = None,
                       shadow_count_only: bool = False) -> dict:
        """kano_verify_combine: OR the gathered word sets of ``nranks`` shards
        and return the results like ``verify`` (column lists global, the
        system row and the shadow pairs of this shard)."""
        out = self._combine_call(
            lambda idx_p, cnt_p, pairs_p, cap, cnt_ref: self.lib.kano_verify_combine(
                self.ctx, c_void_p(gathered_dev_ptr), int(nranks), idx_p, cnt_p, pairs_p, cap,
                cnt_ref),
            "kano_verify_combine", pairs, idx, shadow_count_only)
        if not cross:
            out["user_crosscheck"] = None
        return out

    def _combine_call(self, call, what, pairs, idx, shadow_count_only) -> dict:
        """The combine half's outputs (verify_combine, verify_gather)."""
        n = self.n
        if idx is None:
            idx = np.empty(max(4 * n, 1), dtype=np.int32)
        elif idx.size < 4 * n:
            raise ValueError("idx buffer needs 4*n entries")
        if self._counts is None:
            self._result_slots()
        counts, cnt = self._counts, self._cnt
        shadow = self._shard_shadow
        cap = 0 if pairs is None else pairs.size // 2
        if shadow_count_only:
            cap = -1
        p_idx, p_pairs = self._buf_ptrs(idx, pairs)
        rc = call(p_idx, self._counts_p, p_pairs, int(cap), self._cnt_ref if shadow else None)
        if rc != 0:
            self._chk(rc, what)
        out, o = {}, 0
        for name, k in zip(("all_reachable", "all_isolated", "user_crosscheck",
                            "system_isolation"), counts.tolist()):
            out[name] = idx[o:o + k] if k >= 0 else None
            o += max(k, 0)
        if shadow:
            k = int(cnt.value)
            out["shadow_count"] = k
            if shadow_count_only:
                out["pairs"] = None
            elif pairs is not None and k <= cap:
                out["pairs"] = pairs.reshape(-1)[:2 * k].reshape(k, 2)
            else:
                out["pairs"] = self.shadow_fetch(k)
        return out

    def conflict_raises(self) -> bool:
        v = c_int()
        self._chk(self.lib.kano_conflict(self.ctx, byref(v)), "kano_conflict")
        return bool(v.value)

    def rows_timing(self, reset: bool = False) -> dict:
        """k_rows launch times (HIP events) since the last reset: sum, count,
        min, max (ms); waits for the context's work."""
        out = np.zeros(4, dtype=np.float64)
        self._chk(self.lib.kano_rows_timing(self.ctx, _ptr(out), int(bool(reset))),
                  "kano_rows_timing")
        return dict(sum_ms=float(out[0]), launches=int(out[1]), min_ms=float(out[2]),
                    max_ms=float(out[3]))

    def mfma_timing(self, reset: bool = False) -> dict:
        """k_heavy_mc_mfma per build since the last reset: sum ms, builds,
        algorithmic int8 ops (kano_mfma_timing)."""
        out = np.zeros(4, dtype=np.float64)
        self._chk(self.lib.kano_mfma_timing(self.ctx, _ptr(out), int(bool(reset))),
                  "kano_mfma_timing")
        return dict(sum_ms=float(out[0]), builds=int(out[1]), ops_sum=float(out[2]),
                    ops_last=float(out[3]))

    def set_pipeline(self, on: bool = True) -> None:
        """kano_set_pipeline: each asynchronously completing verify queues the
        next call's prologue behind a gate that the next verify opens (a loop
        of verify calls on the resident inputs).  Call ``settle()`` before a
        device-wide synchronisation outside the engine."""
        self._chk(self.lib.kano_set_pipeline(self.ctx, int(bool(on))), "kano_set_pipeline")

    def settle(self) -> None:
        """kano_settle: no engine work left pending on the device (a queued
        prologue run and put back, the last matrix write finished)."""
        self._chk(self.lib.kano_settle(self.ctx), "kano_settle")

    def gate_timing(self, reset: bool = False) -> dict:
        """kano_gate_timing: how long the pipelined calls' gates held the engine
        stream (its idle time at the step boundary), over the last min(64,
        gates since the last reset) gates; settles first."""
        import ctypes
        g, mean, mx = ctypes.c_int64(0), ctypes.c_double(0.0), ctypes.c_double(0.0)
        self._chk(self.lib.kano_gate_timing(self.ctx, int(bool(reset)), ctypes.byref(g),
                                            ctypes.byref(mean), ctypes.byref(mx)),
                  "kano_gate_timing")
        return dict(gates=int(g.value), mean_us=float(mean.value), max_us=float(mx.value))

    def host_times(self, reset: bool = False) -> dict:
        """kano_verify's host time by phase (us): sums and maxima since the
        last reset (kano_host_times)."""
        out = np.zeros(20, dtype=np.float64)
        self._chk(self.lib.kano_host_times(self.ctx, _ptr(out), int(bool(reset))),
                  "kano_host_times")
        k = ("calls", "front_sum", "back_sum", "wait_sum", "gap_sum", "front_max", "back_max",
             "wait_max", "call_max", "wait1_max", "wait2_max", "wait3_max", "back_launch_max",
             "back_emit_max", "back_tailwait_max", "back_copy_idx_max", "back_copy_pairs_max",
             "back_events_max", "tailwait_sum")
        return {name: float(v) for name, v in zip(k, out)}

    def stage_times(self) -> dict:
        ms = np.zeros(8, dtype=np.float32)
        self._chk(self.lib.kano_stage_times(self.ctx, _ptr(ms)), "kano_stage_times")
        return dict(classes=float(ms[0]), allow=float(ms[1]), select=float(ms[2]),
                    rows=float(ms[3]), shadow=float(ms[4]), build=float(ms[5]),
                    k_rows=float(ms[6]))


def shadow_from_lists(n_lists: int, nbits: int, soff: np.ndarray, slist: np.ndarray,
                      allow_words: np.ndarray, device: int = 0) -> np.ndarray:
    """policy_shadow over explicit per-container policy lists and allow sets
    (the general form of kano_py/kano/algorithm.py:58-80, used when the lists
    are not the ones a single build produced)."""
    lib = nat.load()
    b = DeviceBuild(None, device=device)
    P = allow_words.shape[0]
    soff = np.ascontiguousarray(soff, dtype=np.int64)
    slist = np.ascontiguousarray(slist, dtype=np.int32)
    aw = np.ascontiguousarray(allow_words, dtype=np.uint64)
    cnt = c_int64()
    b._chk(lib.kano_shadow_lists(b.ctx, int(n_lists), int(nbits), int(P), _ptr(soff),
                                 _ptr(slist), _ptr(aw), byref(cnt)), "kano_shadow_lists")
    out = np.zeros((int(cnt.value), 2), dtype=np.int32)
    b._chk(lib.kano_shadow_fetch(b.ctx, _ptr(out)), "kano_shadow_fetch")
    b.close()
    return out
