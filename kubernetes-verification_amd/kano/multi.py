"""One process over G devices: the drop-in API on a row-sharded matrix.

``ReachabilityMatrix.build_matrix`` uses this engine when ``KANO_NGPU`` = G
> 1 (SURVEY.md §8(b) ``kano_init(ngpu)``, §8(e)): a ``kano_group`` (C ABI,
include/kano_hip.h) owns G member contexts, member r on device r (or
``KANO_DEVICES``, comma-separated) holding rows [r0_r, r1_r) of M.  The build
needs no communication; the whole-matrix checks run on the device:

  all_reachable, all_isolated,   each member's [OR | cross | NAND] column
  user_crosscheck                words exchanged (ncclAllGather over xGMI when
  (kano_py/kano/algorithm.py     the devices are distinct, device copies
   :4-42)                        otherwise) and OR-ed on every member
  system_isolation(idx) (:45-55) the row's owner, whichever member it is
  policy_shadow (:58-80)         the members' pairs in rank order (= container
                                 order: the shards are consecutive rows)
  getrow / getcol / [i, j]       the owner / every member's part, in order
  (model.py:171-184)

  add_policies /                 every member's rows (kano_group_add_policies /
  remove_policies (§8(f) rank 4) kano_group_remove_policies)
  two_hop / k_hop / closure      each member's part of the one-hop table,
  (kubesv constraint.py:233-237) gathered, then each member's rows
                                 (kano_group_path)

Shard boundaries are multiples of 64 rows, so a column is the members' word
arrays concatenated.  The engine offers the DeviceBuild methods the drop-in
API calls.

The exchange is RCCL (``ncclAllGather`` over communicators from
``ncclCommInitAll``) whenever the devices are distinct; ``exchange="rccl"`` (or
``KANO_GROUP_RCCL=1``) asks for it even for one member, ``exchange="copy"``
(or ``KANO_GROUP_COPY=1``) for device copies.  A failing RCCL raises: the group
never falls back to copies on its own.
"""
from __future__ import annotations

import os
from ctypes import byref, c_int64, c_void_p
from typing import List, Optional, Tuple

import numpy as np

from . import _native as nat
from ._bits import bool_to_words
from ._engine import DeviceBuild, _ptr
from ._intern import Tables


def shard_bounds(n: int, G: int) -> List[Tuple[int, int]]:
    """Consecutive row ranges, boundaries at multiples of 64 rows."""
    words = (n + 63) >> 6
    out = []
    for r in range(G):
        a = min(n, (words * r // G) << 6)
        b = min(n, (words * (r + 1) // G) << 6)
        out.append((a, b))
    return out


def requested_gpus() -> int:
    try:
        return max(1, int(os.environ.get("KANO_NGPU", "1")))
    except ValueError:
        return 1


def requested_exchange() -> Optional[str]:
    if os.environ.get("KANO_GROUP_RCCL", "") not in ("", "0"):
        return "rccl"
    if os.environ.get("KANO_GROUP_COPY", "") not in ("", "0"):
        return "copy"
    return None


def requested_devices(G: int) -> Optional[List[int]]:
    spec = os.environ.get("KANO_DEVICES")
    if not spec:
        return None
    devs = [int(x) for x in spec.split(",") if x.strip()]
    if len(devs) != G:
        raise ValueError(f"KANO_DEVICES lists {len(devs)} devices for KANO_NGPU={G}")
    return devs


class MultiBuild:
    """A kano_group: G row-shard contexts in one process (see module doc)."""

    def __init__(self, tables: Optional[Tables], ngpu: int, devices: Optional[List[int]] = None,
                 path: str = "auto", build: bool = True, lean: bool = False,
                 exchange: Optional[str] = None):
        self.lib = nat.load()
        self.g = c_void_p()
        G = int(ngpu)
        devs = None
        if devices is not None:
            devs = np.ascontiguousarray(devices, dtype=np.int32)
        # lean: members without the CU-masked write stream (kano_create_lean;
        # the drop-in build_matrix)
        exchange = exchange if exchange is not None else requested_exchange()
        if exchange not in (None, "rccl", "copy"):
            raise ValueError(f"exchange must be 'rccl' or 'copy', not {exchange!r}")
        flags = ((nat.GROUP_LEAN if lean else 0) | (nat.GROUP_RCCL if exchange == "rccl" else 0) |
                 (nat.GROUP_COPY if exchange == "copy" else 0))
        rc = self.lib.kano_group_create_ex(G, _ptr(devs), flags, byref(self.g))
        if rc != 0:
            self.g = c_void_p()
            why = self.lib.kano_group_last_error(None)
            raise nat.KanoNativeError(f"kano_group_create({G}) failed (rc={rc}): "
                                      f"{why.decode(errors='replace') if why else ''}")
        self.G = G
        self.devices = list(devices) if devices is not None else list(range(G))
        self.lean = lean
        self.exchange = exchange
        self.path = path
        self.tables = tables
        self.row_span = None
        self.bounds = shard_bounds(tables.n, G) if tables is not None else None
        info = np.zeros(2, dtype=np.int32)
        self.lib.kano_group_info(self.g, _ptr(info))
        self.mode = {1: "rccl all-gather", 2: "device copies"}[int(info[1])]
        self.members: List[DeviceBuild] = []
        for r in range(G):
            ctx = c_void_p()
            self._chk(self.lib.kano_group_member(self.g, r, byref(ctx)), "kano_group_member")
            m = DeviceBuild.adopt(ctx, device=int(devices[r]) if devices is not None else r,
                                  path=path)
            self.members.append(m)
        self.device = self.members[0].device
        self._idx = None
        if tables is not None:   # (None: the caller uploads, then builds)
            self.upload(tables)
            if build:
                self.build(path)

    def upload(self, t: Tables) -> None:
        """kano_group_upload: the tables to every member at once, member r's
        row shard set (the members' own threads)."""
        self.tables = t
        self.bounds = shard_bounds(t.n, self.G)
        pv = np.ascontiguousarray(t.pod_val, dtype=np.int32)
        ex = [None] * 4
        E = 0
        if getattr(t, "expr_col", None) is not None and len(t.expr_col):
            ex = [np.ascontiguousarray(a, dtype=d) for a, d in (
                (t.expr_col, np.int32), (t.expr_op, np.int32), (t.expr_off, np.int64),
                (t.expr_val, np.int32))]
            E = len(ex[0])
        arrs = [np.ascontiguousarray(a, dtype=d) for a, d in (
            (t.sel_off, np.int64), (t.sel_col, np.int32), (t.sel_val, np.int32),
            (t.alw_off, np.int64), (t.alw_col, np.int32), (t.alw_val, np.int32))]
        b = np.ascontiguousarray(np.asarray(self.bounds, dtype=np.int64).reshape(-1))
        self._chk(self.lib.kano_group_upload(self.g, t.n, t.ncols, _ptr(pv), E,
                                             *[_ptr(a) for a in ex], t.P,
                                             *[_ptr(a) for a in arrs], _ptr(b)),
                  "kano_group_upload")
        for m, (a, bb) in zip(self.members, self.bounds):
            m.tables = t
            m.row_span = None if (a, bb) == (0, t.n) else (a, bb)

    # -- plumbing -------------------------------------------------------
    def _chk(self, rc, what):
        if rc != 0:
            raw = self.lib.kano_group_last_error(self.g) if self.g else b""
            raise nat.KanoNativeError(f"{what} failed (rc={rc}): "
                                      f"{raw.decode(errors='replace') if raw else ''}")

    def close(self):
        if self.g:
            for m in self.members:
                m.close()                   # (adopted: drops the handle; the group owns it)
            self.lib.kano_group_destroy(self.g)
            self.g = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n(self) -> int:
        return self.tables.n

    @property
    def W(self) -> int:
        return (self.tables.n + 63) >> 6

    is_shard = False

    def owner(self, i: int) -> int:
        for r, (a, b) in enumerate(self.bounds):
            if a <= i < b:
                return r
        raise IndexError("row out of range")

    def build(self, path: Optional[str] = None) -> None:
        """kano_group_build: every member's row shard at once."""
        self._chk(self.lib.kano_group_build(self.g, nat.PATHS[path or self.path]),
                  "kano_group_build")

    def set_groups(self, gid: np.ndarray, ngroups: int = 0) -> None:
        """kano_group_set_groups: the pods' group ids on every member (then
        ``verify(gid="stored")``)."""
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        if gid.shape[0] != self.n:
            raise ValueError("gid must have one entry per pod")
        self._chk(self.lib.kano_group_set_groups(self.g, _ptr(gid), int(ngroups)),
                  "kano_group_set_groups")

    def info(self) -> dict:
        infos = [m.info() for m in self.members]
        out = dict(infos[0])
        out["ROW0"], out["ROW1"] = 0, self.n
        for k in ("U", "NNZ_SEL", "HEAVY", "WORK_ITEMS"):
            out[k] = sum(i[k] for i in infos)
        out["MAXSEL"] = max(i["MAXSEL"] for i in infos)
        return out

    # -- whole-matrix checks on the device ----------------------------------
    def _lists(self, counts, idx):
        out, o = {}, 0
        for r, name in enumerate(("all_reachable", "all_isolated", "user_crosscheck",
                                  "system_isolation")):
            k = int(counts[r])
            out[name] = idx[o:o + k] if k >= 0 else None
            o += max(k, 0)
        return out

    def _idx_buf(self):
        if self._idx is None or self._idx.size < 4 * max(self.n, 1):
            self._idx = np.empty(4 * max(self.n, 1), dtype=np.int32)
        return self._idx

    def checks(self, gid: Optional[np.ndarray] = None, sys_row: int = -1) -> dict:
        """kano_group_checks: the column lists over every member's rows (and
        the owner's system row when sys_row >= 0)."""
        counts = np.zeros(4, dtype=np.int64)
        idx = self._idx_buf()
        g = None if gid is None else np.ascontiguousarray(gid, dtype=np.int32)
        self._chk(self.lib.kano_group_checks(self.g, _ptr(g), 0, int(sys_row), _ptr(idx),
                                             counts.ctypes.data), "kano_group_checks")
        return {k: (None if v is None else v.copy()) for k, v in self._lists(counts, idx).items()}

    def col_checks(self) -> Tuple[np.ndarray, np.ndarray]:
        r = self.checks()
        n = self.n
        reach = np.zeros(n, bool)
        reach[r["all_reachable"]] = True
        reached = np.ones(n, bool)
        reached[r["all_isolated"]] = False
        return bool_to_words(reach), bool_to_words(reached)

    def crosscheck(self, gid: np.ndarray) -> np.ndarray:
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        if gid.shape[0] != self.n:
            raise ValueError("gid must have one entry per pod")
        r = self.checks(gid)
        bits = np.zeros(self.n, bool)
        bits[r["user_crosscheck"]] = True
        return bool_to_words(bits)

    def verify(self, gid=None, sys_row: int = 0, shadow: bool = True,
               pairs: Optional[np.ndarray] = None, idx: Optional[np.ndarray] = None,
               path: Optional[str] = None, shadow_count_only: bool = False) -> dict:
        """kano_group_verify: build + every check over all G members (as
        DeviceBuild.verify)."""
        n = self.n
        if idx is None:
            idx = np.empty(max(4 * n, 1), dtype=np.int32)
        ngroups = 0
        stored = isinstance(gid, str) and gid == "stored"
        if stored:
            g, ngroups = None, nat.STORED_GROUPS
        else:
            g = None if gid is None else np.ascontiguousarray(gid, dtype=np.int32)
        counts = np.zeros(4, dtype=np.int64)
        cnt = c_int64(0)
        cap = 0 if pairs is None else pairs.size // 2
        if shadow_count_only:
            cap = -1
        with_shadow = 0 if not shadow else (2 if shadow_count_only else 1)
        pth = nat.PATHS[path or self.path]
        self._chk(self.lib.kano_group_verify(self.g, pth, _ptr(g), ngroups, int(sys_row),
                                             with_shadow,
                                             _ptr(idx), counts.ctypes.data, _ptr(pairs), int(cap),
                                             byref(cnt) if shadow else None), "kano_group_verify")
        out = self._lists(counts, idx)
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
                out["pairs"] = np.concatenate([m.shadow_fetch(m.shadow_count())
                                               for m in self.members]).reshape(-1, 2)
        return out

    def shadow(self) -> np.ndarray:
        """policy_shadow's pairs: each member's (its containers), rank order."""
        parts = [m.shadow() for m in self.members]
        return np.concatenate(parts).reshape(-1, 2) if parts else np.zeros((0, 2), np.int32)

    def conflict_raises(self) -> bool:
        return any(m.conflict_raises() for m in self.members)

    # -- matrix access: owners --------------------------------------------
    def rows(self, r0: int, nrows: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        if out is None:
            out = np.zeros((nrows, self.W), dtype=np.uint64)
        for m, (a, b) in zip(self.members, self.bounds):
            lo, hi = max(a, r0), min(b, r0 + nrows)
            if lo < hi:
                m.rows(lo, hi - lo, out[lo - r0:hi - r0])
        return out

    def put_rows(self, r0: int, words: np.ndarray) -> None:
        words = np.ascontiguousarray(words, dtype=np.uint64).reshape(-1, self.W)
        for m, (a, b) in zip(self.members, self.bounds):
            lo, hi = max(a, r0), min(b, r0 + words.shape[0])
            if lo < hi:
                m.put_rows(lo, words[lo - r0:hi - r0])

    def col(self, j: int) -> np.ndarray:
        """Column j: every member's rows' bits (64-row aligned shards)."""
        parts = [m.col(j) for m, (a, b) in zip(self.members, self.bounds) if b > a]
        return np.concatenate(parts)[: self.W] if parts else np.zeros(self.W, np.uint64)

    def get_bit(self, i: int, j: int) -> int:
        return self.members[self.owner(int(i))].get_bit(i, j)

    def set_bit(self, i: int, j: int, value) -> None:
        self.members[self.owner(int(i))].set_bit(i, j, value)

    def export_rows(self, r0: int, nrows: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        nb = (self.n + 7) >> 3
        if out is None:
            out = np.empty((max(nrows, 0), nb), dtype=np.uint8)
        for m, (a, b) in zip(self.members, self.bounds):
            lo, hi = max(a, r0), min(b, r0 + nrows)
            if lo < hi:
                m.export_rows(lo, hi - lo, out[lo - r0:hi - r0])
        return out

    def import_rows(self, r0: int, rows: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.uint8)
        for m, (a, b) in zip(self.members, self.bounds):
            lo, hi = max(a, r0), min(b, r0 + rows.shape[0])
            if lo < hi:
                m.import_rows(lo, rows[lo - r0:hi - r0])

    # -- build side effects (Container / Policy lists) ------------------------
    def classes(self) -> np.ndarray:
        """Row class of every pod, ids made global (member r's classes offset
        by the classes of members < r)."""
        out = np.full(self.n, -1, dtype=np.int32)
        base = 0
        for m, (a, b) in zip(self.members, self.bounds):
            c = m.classes()
            out[a:b] = c[a:b] + base
            base += m.info()["U"]
        return out

    def select_csr(self) -> Tuple[np.ndarray, np.ndarray]:
        offs, pols, base = [np.zeros(1, np.int64)], [], 0
        for m in self.members:
            off, pol = m.select_csr()
            offs.append(off[1:] + base)
            pols.append(pol)
            base += int(off[-1])
        return np.concatenate(offs), (np.concatenate(pols) if pols else np.zeros(0, np.int32))

    def allow_csr(self) -> Tuple[np.ndarray, np.ndarray]:
        return self.members[0].allow_csr()   # the column side is whole on every member

    def policy_sets(self, p: int, sel: bool = True, allow: bool = True):
        s = None
        if sel:
            s = np.zeros(self.W, dtype=np.uint64)
            for m in self.members:
                s |= m.policy_sets(p, True, False)[0]
        a = self.members[0].policy_sets(p, False, True)[1] if allow else None
        return s, a

    # -- incremental updates -------------------------
    def add_policies(self, xval: np.ndarray, sel_csr, alw_csr) -> int:
        """kano_group_add_policies: every member's rows; returns the first
        new engine id (equal on every member)."""
        so, sc, sv = (np.ascontiguousarray(a, dtype=d) for a, d in
                      zip(sel_csr, (np.int64, np.int32, np.int32)))
        ao, ac, av = (np.ascontiguousarray(a, dtype=d) for a, d in
                      zip(alw_csr, (np.int64, np.int32, np.int32)))
        xv = np.ascontiguousarray(xval, dtype=np.int32)
        first = c_int64(0)
        self._chk(self.lib.kano_group_add_policies(
            self.g, int(so.shape[0] - 1), int(xv.shape[0]), _ptr(xv), _ptr(so), _ptr(sc),
            _ptr(sv), _ptr(ao), _ptr(ac), _ptr(av), byref(first)), "kano_group_add_policies")
        return int(first.value)

    def remove_policies(self, ids) -> None:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.int64).reshape(-1))
        self._chk(self.lib.kano_group_remove_policies(self.g, int(a.shape[0]), _ptr(a)),
                  "kano_group_remove_policies")

    def added_policy_sets(self, eid: int) -> Tuple[np.ndarray, np.ndarray]:
        # (the added policies' sets cover every pod on every member)
        return self.members[0].added_policy_sets(eid)

    # -- multi-hop reachability ------------------------
    @classmethod
    def empty(cls, n: int, ngpu: int, devices: Optional[List[int]] = None) -> "MultiBuild":
        """A group holding an n x n matrix in the same row shards and no
        policies (the target of path_from)."""
        z64 = np.zeros(1, np.int64)
        e = np.zeros(0, np.int32)
        t = Tables(int(n), 0, np.zeros((0, int(n)), np.int32), z64, e, e, z64, e, e)
        return cls(t, ngpu, devices=devices, lean=True, exchange="copy")

    def path_from(self, src: "MultiBuild", hops: int = 2, mode: str = "auto") -> dict:
        """This group's rows := the multi-hop reachability of src's row-sharded
        matrix (kano_group_path; kubesv/kubesv/constraint.py:233-237): one
        exchange of the members' one-hop table parts over src's transport."""
        if not isinstance(src, MultiBuild) or src.G != self.G or src.devices != self.devices:
            raise ValueError("path_from needs a group over the same devices")
        info = np.zeros(6, dtype=np.int64)
        self._chk(self.lib.kano_group_path(src.g, self.g, int(hops), nat.PATHS[mode], _ptr(info)),
                  "kano_group_path")
        keys = ("steps", "steps_run", "mfma_steps", "row_classes", "col_classes", "identity")
        return {k: int(v) for k, v in zip(keys, info)}

    # -- measurement ------------------------------------------------------------
    def exchange_timing(self, enable: Optional[bool] = None, reset: bool = False) -> dict:
        """The verify exchange's time on member 0's stream (HIP events around
        the all-gather or the copies; enable=True switches it on)."""
        out = np.zeros(3, dtype=np.float64)
        self._chk(self.lib.kano_group_exchange_timing(
            self.g, -1 if enable is None else int(bool(enable)), _ptr(out), int(reset)),
            "kano_group_exchange_timing")
        return {"calls": int(out[0]), "total_ms": float(out[1]), "max_ms": float(out[2]),
                "avg_ms": float(out[1] / out[0]) if out[0] else None}
