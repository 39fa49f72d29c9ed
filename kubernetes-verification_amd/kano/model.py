"""Kano data model, drop-in for ``kano.model`` of kano_py.

Same names, fields and behaviour as kano_py/kano/model.py; the difference is
where the state lives.  ``ReachabilityMatrix.build_matrix`` interns the
labels (kano/_intern.py) and builds the matrix on the GPU through
libkano_hip.so (kano/_engine.py); the matrix stays in HBM and the Python
objects are views of it:

* ``m.matrix[i]`` / ``m.getrow(i)`` are *live* rows (reads and writes go to the
  device), like the reference's list of bitarrays (model.py:167-178);
* ``m.getcol(j)`` gathers a column on the device (model.py:180-184);
* ``Policy.working_select_set`` / ``working_allow_set`` are filled by the
  build with bitarray-compatible sets fetched on first use (model.py:119-121);
* ``Container.select_policies`` / ``allow_policies`` receive the build's
  appends lazily, in build order, so repeated builds accumulate exactly as in
  the reference (model.py:158-163, quirk Q5).

There is no CPU fallback: without the HIP library or a GPU the build raises
``KanoNativeError``.
"""
from __future__ import annotations

import gc
import threading

from abc import abstractmethod
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple, TypeVar

try:                                    # the reference imports typing_extensions
    from typing_extensions import Protocol
except ImportError:                     # pragma: no cover
    from typing import Protocol

import itertools

import numpy as np

from ._bits import BitArray, bool_to_words, words_to_bool
from . import _native

__all__ = [
    "Container", "PolicySelect", "PolicyAllow", "PolicyDirection", "PolicyIngress",
    "PolicyEgress", "PolicyProtocol", "LabelRelation", "DefaultEqualityLabelRelation",
    "Policy", "ReachabilityMatrix", "BitArray", "bitarray", "KanoNativeError",
    "LabelExpression", "In", "NotIn", "Exists", "DoesNotExist",
]

bitarray = BitArray
KanoNativeError = _native.KanoNativeError


_BUILD_IDS = itertools.count(1)


class _BuildLists:
    """Host-side, lazily fetched view of one build's per-container lists.
    ``bid`` names the build's segment of every container's accumulated
    lists (quirk Q5: each build appends after the previous builds' entries)."""

    def __init__(self, engine, containers=None):
        self._engine = engine
        self._sel = None
        self._alw = None
        self.bid = next(_BUILD_IDS)
        # the build's container list: a container's pending entry is this
        # object itself (no per-container allocation), its row index found
        # here on first use
        self._containers = containers
        self._pos = None
        self._dups = None

    def position(self, c, k: int = 0) -> int:
        if self._pos is None:
            pos: Dict[int, int] = {}
            dups: Dict[int, List[int]] = {}
            for i, x in enumerate(self._containers):
                j = pos.setdefault(id(x), i)
                if j != i:
                    dups.setdefault(id(x), [j]).append(i)
            self._pos, self._dups = pos, dups
        d = self._dups.get(id(c))
        return d[k] if d is not None else self._pos[id(c)]

    def select_list(self, i: int) -> List[int]:
        if self._sel is None:
            cls = self._engine.classes()
            off, pol = self._engine.select_csr()
            self._sel = (cls, off, pol)
        cls, off, pol = self._sel
        c = cls[i]
        return pol[off[c]:off[c + 1]].tolist()

    def allow_list(self, i: int) -> List[int]:
        if self._alw is None:
            aoff, pods = self._engine.allow_csr()
            P = aoff.shape[0] - 1
            pol = np.repeat(np.arange(P, dtype=np.int32), np.diff(aoff))
            order = np.argsort(pods, kind="stable")
            n = self._engine.n
            cnt = np.bincount(pods, minlength=n)
            off = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(cnt, out=off[1:])
            self._alw = (off, pol[order])
        off, pol = self._alw
        return pol[off[i]:off[i + 1]].tolist()


class _Renumber:
    """ReachabilityMatrix.remove_policies on a container's lists: within the
    segment build ``bid`` appended, drop the removed policy indices and
    renumber the rest (what that build over the updated policy list would
    have appended); other builds' entries (Q5) are left alone."""

    __slots__ = ("gone", "lo", "bid")

    def __init__(self, gone: np.ndarray, bid: int):
        self.gone = gone
        self.lo = int(gone[0])
        self.bid = bid

    def apply_list(self, lst: List[int]) -> None:
        lo = self.lo
        if any(x >= lo for x in lst):
            arr = np.asarray(lst, dtype=np.int64)
            keep = arr[~np.isin(arr, self.gone)]
            lst[:] = (keep - np.searchsorted(self.gone, keep, side="right")).tolist()

    def apply(self, c: "Container") -> None:
        seg = c._seg.get(self.bid)
        if seg is None:
            return
        for which, lst in ((0, c._sel), (2, c._alw)):
            a, b = seg[which], seg[which + 1]
            part = lst[a:b]
            self.apply_list(part)
            lst[a:b] = part
            c._shift(which, b, len(part) - (b - a), self.bid)


class Container:
    """A container (kano_py/kano/model.py:11-25).  Dataclass-equivalent:
    fields ``name, labels, select_policies, allow_policies``; the two lists
    receive each build's appends lazily (see module docstring)."""

    __slots__ = ("name", "labels", "_sel", "_alw", "_pending", "_seg", "__weakref__")
    __match_args__ = ("name", "labels", "select_policies", "allow_policies")

    def __init__(self, name: str, labels: Dict[str, str],
                 select_policies: Optional[List[int]] = None,
                 allow_policies: Optional[List[int]] = None):
        self.name = name
        self.labels = labels
        self._sel = [] if select_policies is None else select_policies
        self._alw = [] if allow_policies is None else allow_policies
        self._pending: List[tuple] = []
        # build id -> [sel start, sel end, allow start, allow end]: where each
        # build's appends sit in the accumulated lists
        self._seg: Dict[int, List[int]] = {}

    def _flush(self) -> None:
        if self._pending:
            pend, self._pending = self._pending, []
            seen: Dict[int, int] = {}
            for e in pend:
                if type(e) is tuple:               # (a policy removal, applied lazily)
                    e[0].apply(self)
                    continue
                # a build's entry: the k-th for this build is this container's
                # k-th position in the build's container list
                lists = e
                k = seen.get(lists.bid, 0)
                seen[lists.bid] = k + 1
                i = lists.position(self, k)
                s0, a0 = len(self._sel), len(self._alw)
                self._sel.extend(lists.select_list(i))
                self._alw.extend(lists.allow_list(i))
                self._seg[lists.bid] = [s0, len(self._sel), a0, len(self._alw)]

    def _shift(self, which: int, at: int, delta: int, bid: int) -> None:
        """Segment bid's list (0 select, 2 allow) grew by delta at position
        at: move its end and every later segment."""
        if delta == 0:
            return
        for k, seg in self._seg.items():
            if k == bid:
                seg[which + 1] += delta
            elif seg[which] >= at:
                seg[which] += delta
                seg[which + 1] += delta

    def _seg_append(self, bid: int, which: int, value: int) -> None:
        """An incremental add: the build bid over the extended policy list
        would have appended value at the end of its segment."""
        self._flush()
        lst = self._sel if which == 0 else self._alw
        seg = self._seg.get(bid)
        if seg is None:
            lst.append(value)
            return
        at = seg[which + 1]
        lst.insert(at, value)
        self._shift(which, at, 1, bid)

    @property
    def select_policies(self) -> List[int]:
        self._flush()
        return self._sel

    @select_policies.setter
    def select_policies(self, v: List[int]) -> None:
        self._flush()
        self._sel = v
        self._seg = {}       # a replaced list has no build segments

    @property
    def allow_policies(self) -> List[int]:
        self._flush()
        return self._alw

    @allow_policies.setter
    def allow_policies(self, v: List[int]) -> None:
        self._flush()
        self._alw = v
        self._seg = {}

    def getValueOrDefault(self, key: str, value: str):
        if key in self.labels:
            return self.labels[key]
        return value

    def getLabels(self):
        return self.labels

    def __repr__(self) -> str:
        return (f"Container(name={self.name!r}, labels={self.labels!r}, "
                f"select_policies={self.select_policies!r}, "
                f"allow_policies={self.allow_policies!r})")

    def __eq__(self, other):
        if other.__class__ is not self.__class__:
            return NotImplemented
        return ((self.name, self.labels, self.select_policies, self.allow_policies) ==
                (other.name, other.labels, other.select_policies, other.allow_policies))

    __hash__ = None


class LabelExpression:
    """Kubernetes matchExpressions requirement as a PolicySelect / PolicyAllow
    value (not in kano_py).  Semantics follow the
    label-selector requirements kubesv adapts (kubesv/kubesv/model.py:127-160,
    operators In / NotIn / Exists / DoesNotExist): In needs the key with a
    listed value, NotIn matches an absent key or an unlisted value, Exists
    needs the key, DoesNotExist its absence.  Unlike a plain value, the term
    is evaluated whether or not any container carries the key (no quirk Q1).
    Values compare by Python ==, like the default matcher."""

    op = -1

    def matches(self, labels: Dict, key) -> bool:
        raise NotImplementedError

    def __eq__(self, other):
        return type(other) is type(self) and getattr(other, "values", None) == getattr(
            self, "values", None)

    def __hash__(self):
        return hash((type(self).__name__, tuple(getattr(self, "values", ()))))

    def __repr__(self):
        v = getattr(self, "values", None)
        return f"{type(self).__name__}({v!r})" if v is not None else f"{type(self).__name__}()"


def _listed(v, values) -> bool:
    return any(v == x for x in values)


class In(LabelExpression):
    op = 0

    def __init__(self, values):
        self.values = list(values)

    def matches(self, labels, key):
        return key in labels and _listed(labels[key], self.values)


class NotIn(LabelExpression):
    op = 1

    def __init__(self, values):
        self.values = list(values)

    def matches(self, labels, key):
        return key not in labels or not _listed(labels[key], self.values)


class Exists(LabelExpression):
    op = 2

    def matches(self, labels, key):
        return key in labels


class DoesNotExist(LabelExpression):
    op = 3

    def matches(self, labels, key):
        return key not in labels


@dataclass
class PolicySelect:
    labels: Dict[str, str]


@dataclass
class PolicyAllow:
    labels: Dict[str, str]


@dataclass
class PolicyDirection:
    # true for ingress, false for egress (model.py:38-47)
    direction: bool

    def is_ingress(self) -> bool:
        return self.direction

    def is_egress(self) -> bool:
        return not self.direction


PolicyIngress = PolicyDirection(True)
PolicyEgress = PolicyDirection(False)


@dataclass
class PolicyProtocol:
    protocols: List[str]


T = TypeVar("T")


class LabelRelation(Protocol[T]):
    @abstractmethod
    def match(self, rule: T, value: T) -> bool:
        raise NotImplementedError


class DefaultEqualityLabelRelation(LabelRelation):
    def match(self, rule: Any, value: Any) -> bool:
        return rule == value


class _LazySet(BitArray):
    """Policy.working_select_set / working_allow_set of one build, fetched from
    the device on first use, then an ordinary mutable bit vector."""

    __slots__ = ("_src",)

    def __init__(self, engine, p: int, which: str):
        self._src = (engine, p, which)
        self._n = engine.n
        self._wd = None

    def _words(self) -> np.ndarray:
        if self._wd is None:
            engine, p, which = self._src
            s, a = engine.policy_sets(p, sel=(which == "sel"), allow=(which == "allow"))
            self._wd = s if which == "sel" else a
        return self._wd


@dataclass
class Policy:
    name: str
    selector: PolicySelect
    allow: PolicyAllow
    direction: PolicyDirection
    protocol: PolicyProtocol
    matcher: LabelRelation[str] = DefaultEqualityLabelRelation()
    working_select_set: Any = None
    working_allow_set: Any = None

    @property
    def working_selector(self):
        # egress: (select = selector, allow = allow); ingress swaps (model.py:82-93)
        if self.is_egress():
            return self.selector
        return self.allow

    @property
    def working_allow(self):
        if self.is_egress():
            return self.allow
        return self.selector

    # Per-container predicates kept for API parity (model.py:95-111); the build
    # evaluates the same predicate on the GPU over interned labels.
    # (LabelExpression values, an extension, are evaluated on their own)
    def select_policy(self, container: Container) -> bool:
        return self._pred(self.working_selector.labels, container)

    def allow_policy(self, container: Container) -> bool:
        return self._pred(self.working_allow.labels, container)

    def _pred(self, sl, container) -> bool:
        for k, rule in sl.items():
            if isinstance(rule, LabelExpression) and not rule.matches(container.labels, k):
                return False
        for k, v in container.labels.items():
            if k in sl.keys() and not isinstance(sl[k], LabelExpression) and \
                    not self.matcher.match(sl[k], v):
                return False
        return True

    def is_ingress(self):
        return self.direction.is_ingress()

    def is_egress(self):
        return self.direction.is_egress()

    def store_bcp(self, select_set, allow_set):
        self.working_select_set = select_set
        self.working_allow_set = allow_set


class _Row(BitArray):
    """A live row of a device-resident matrix (model.py:177-178 aliasing)."""

    __slots__ = ("_m", "_i")

    def __init__(self, m: "ReachabilityMatrix", i: int):
        self._m = m
        self._i = i
        self._n = m.container_size

    def _words(self) -> np.ndarray:
        return self._m._engine.rows(self._i, 1)[0]

    def _store(self, words: np.ndarray) -> None:
        self._m._engine.put_rows(self._i, words.reshape(1, -1))

    def __setitem__(self, key, value):
        if isinstance(key, slice):
            return BitArray.__setitem__(self, key, value)
        i = self._norm(key)
        self._m._engine.set_bit(self._i, i, value)


class _Rows:
    """``ReachabilityMatrix.matrix``: a list-like of live rows."""

    def __init__(self, m: "ReachabilityMatrix"):
        self._m = m

    def __len__(self):
        return self._m.container_size

    def _norm(self, i: int) -> int:
        n = self._m.container_size
        i = int(i)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("list index out of range")
        return i

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        return _Row(self._m, self._norm(i))

    def __setitem__(self, i, row):
        i = self._norm(i)
        b = row if isinstance(row, BitArray) else BitArray(row)
        if len(b) != self._m.container_size:
            raise ValueError("row length must equal container_size")
        self._m._engine.put_rows(i, b.words().reshape(1, -1))

    def __iter__(self):
        for i in range(len(self)):
            yield _Row(self._m, i)


class ReachabilityMatrix:
    """Container-to-container reachability (kano_py/kano/model.py:124-184),
    resident in HBM."""

    @staticmethod
    def build_matrix(containers: List[Container], policies: List[Policy]):
        from ._engine import DeviceBuild
        from ._intern import intern
        from .multi import MultiBuild, requested_devices, requested_gpus
        # (the cyclic GC paused over the bulk object work: with 10^5 live
        # containers each full collection walks them all -- 0.18 s a pass on
        # C3 -- and the per-policy objects below used to trigger several)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            # the engine's contexts are made on a second thread while this
            # one interns (the native calls release the GIL): ~7 ms per
            # context off the cold call
            G = requested_gpus()
            made: Dict[str, Any] = {}

            def make():
                try:
                    made["e"] = (MultiBuild(None, G, devices=requested_devices(G), lean=True)
                                 if G > 1 else DeviceBuild(None, lean=True))
                except BaseException as exc:   # noqa: BLE001 (re-raised below)
                    made["x"] = exc
            maker = threading.Thread(target=make, name="kano-create")
            maker.start()
            try:
                tables = intern(containers, policies)
            except BaseException:
                maker.join()
                if "e" in made:
                    made["e"].close()
                raise
            maker.join()
            if "x" in made:
                raise made["x"]
            engine = made["e"]
            try:
                engine.upload(tables)
                engine.build()
            except BaseException:
                engine.close()           # (the contexts and their device memory now)
                raise
            for p, pol in enumerate(policies):
                pol.store_bcp(_LazySet(engine, p, "sel"), _LazySet(engine, p, "allow"))
            # (the build's order, snapshotted: a caller reordering its list
            # afterwards must not move the lists between containers)
            lists = _BuildLists(engine, list(containers))
            for i, c in enumerate(containers):
                if isinstance(c, Container):
                    c._pending.append(lists)
                else:                        # foreign container type: materialise now
                    c.select_policies.extend(lists.select_list(i))
                    c.allow_policies.extend(lists.allow_list(i))
        finally:
            if gc_was:
                gc.enable()
        m = ReachabilityMatrix.__new__(ReachabilityMatrix)
        m.container_size = len(containers)
        m._engine = engine
        # kept so that policy_shadow can tell whether it is handed the very
        # lists this build produced (then it runs on the device's class lists)
        m._containers = containers
        m._policies = policies
        m._ncontainers = len(containers)
        m._lists = lists
        m._bid = lists.bid
        return m

    def __init__(self, container_size: int, matrix: Any) -> None:
        """Wrap an explicit matrix (a sequence of container_size bit rows) as the
        reference constructor does (model.py:167-169); it is uploaded to HBM."""
        from ._engine import DeviceBuild
        from ._intern import Tables
        n = int(container_size)
        z64 = np.zeros(1, np.int64)
        empty = np.zeros(0, np.int32)
        t = Tables(n, 0, np.zeros((0, n), np.int32), z64, empty, empty, z64, empty, empty)
        self.container_size = n
        self._engine = DeviceBuild(t)
        self._containers = None
        self._policies = None
        self._ncontainers = n
        self._lists = None
        rows = list(matrix)
        if len(rows) != n:
            raise ValueError("matrix must have container_size rows")
        if n:
            W = (n + 63) >> 6
            words = np.zeros((n, W), dtype=np.uint64)
            for i, r in enumerate(rows):
                b = r if isinstance(r, BitArray) else BitArray(r)
                words[i] = b.words()[:W] if len(b) == n else _fit(b, n)
            self._engine.put_rows(0, words)

    @property
    def matrix(self) -> _Rows:
        return _Rows(self)

    def __setitem__(self, key, value):
        i, j = key
        n = self.container_size
        i = int(i) + n if int(i) < 0 else int(i)
        j = int(j) + n if int(j) < 0 else int(j)
        if not (0 <= i < n and 0 <= j < n):
            raise IndexError("bitarray index out of range")
        self._engine.set_bit(i, j, value)

    def __getitem__(self, key):
        i, j = key
        n = self.container_size
        i = int(i) + n if int(i) < 0 else int(i)
        j = int(j) + n if int(j) < 0 else int(j)
        if not (0 <= i < n and 0 <= j < n):
            raise IndexError("bitarray index out of range")
        return self._engine.get_bit(i, j)

    def getrow(self, index):
        return self.matrix[index]

    def getcol(self, index):
        n = self.container_size
        j = int(index)
        if not 0 <= j < n:
            raise IndexError("bitarray index out of range")
        if getattr(self._engine, "is_shard", False):
            r0, r1 = self._engine.row_span
            raise ValueError(f"matrix holds only rows [{r0}, {r1}) of {n}: a column needs "
                             "every row")
        return BitArray.from_words(self._engine.col(j), n)

    # engine access for kano.algorithm
    @property
    def engine(self):
        return self._engine

    # ---- incremental policy updates ----------
    # Not in kano_py, whose only way to change the policy set is another
    # build_matrix call.  After add_policies / remove_policies the matrix,
    # every container's select_policies / allow_policies and the policies'
    # working sets are what build_matrix(containers, updated policies) gives
    # (model.py:125-165); the device writes only the rows the changed
    # policies select.  The build's policy list is updated in place.

    def _check_inc(self):
        if getattr(self, "_policies", None) is None:
            raise TypeError("incremental updates need a matrix from build_matrix")
        if getattr(self, "_eids", None) is None:
            self._eids = list(range(len(self._policies)))

    def add_policies(self, new_policies: List["Policy"]) -> None:
        from ._intern import intern_more
        from ._bits import set_bit_indices
        self._check_inc()
        new_policies = list(new_policies)
        for pol in new_policies:          # allow=None raises here, as the build does
            pol.working_selector.labels
            pol.working_allow.labels
        eng = self._engine
        n = self.container_size
        xval, sel, alw = intern_more(eng.tables, new_policies)
        first = eng.add_policies(xval, sel, alw)
        cs, ps = self._containers, self._policies
        for k, pol in enumerate(new_policies):
            eid = first + k
            idx = len(ps)
            s, a = eng.added_policy_sets(eid)
            pol.store_bcp(BitArray.from_words(s, n), BitArray.from_words(a, n))
            for i in set_bit_indices(s, n).tolist():
                if isinstance(cs[i], Container):
                    cs[i]._seg_append(self._bid, 0, idx)
                else:
                    cs[i].select_policies.append(idx)
            for j in set_bit_indices(a, n).tolist():
                if isinstance(cs[j], Container):
                    cs[j]._seg_append(self._bid, 2, idx)
                else:
                    cs[j].allow_policies.append(idx)
            ps.append(pol)
            self._eids.append(eid)
        self._lists = None

    def remove_policies(self, indices) -> None:
        self._check_inc()
        ps, cs = self._policies, self._containers
        idx = sorted({int(k) + len(ps) if int(k) < 0 else int(k) for k in indices})
        if any(k < 0 or k >= len(ps) for k in idx):
            raise IndexError("list index out of range")
        if not idx:
            return
        self._engine.remove_policies([self._eids[k] for k in idx])
        # the lists drop the removed indices and renumber the rest (lazily,
        # in order with the build's own pending lists)
        op = _Renumber(np.asarray(idx, dtype=np.int64), self._bid)
        for c in cs:
            if isinstance(c, Container):
                c._pending.append((op, -1))
            else:
                op.apply_list(c.select_policies)
                op.apply_list(c.allow_policies)
        for k in reversed(idx):
            del ps[k]
            del self._eids[k]
        self._lists = None

    # ---- on-disk / tooling format -------------
    # Not in kano_py: its rows are bitarrays (model.py:136-139), and this
    # format is their bytes.  File: b"KANOMAT1", then n, r0, r1, row_bytes as
    # little-endian u64, then rows r0..r1-1, each bitarray(row).tobytes()
    # (big-endian bit order, ceil(n/8) bytes, pad bits zero).  A row shard
    # (multi-GPU, kano/shard.py) writes its own range; shard files of one
    # matrix concatenate in row order.
    MAGIC = b"KANOMAT1"

    def row_bytes(self, r0: int = 0, nrows: Optional[int] = None) -> np.ndarray:
        """Rows [r0, r0+nrows) as bitarray bytes, shape (nrows, ceil(n/8))."""
        n = self.container_size
        if nrows is None:
            nrows = n - r0
        return self._engine.export_rows(r0, nrows)

    def save(self, path: str, rows: Optional[Tuple[int, int]] = None,
             chunk_bytes: int = 64 << 20) -> None:
        n = self.container_size
        r0, r1 = rows if rows is not None else (0, n)
        nb = (n + 7) >> 3
        step = max(1, chunk_bytes // max(nb, 1))
        with open(path, "wb") as f:
            f.write(self.MAGIC)
            f.write(np.array([n, r0, r1, nb], dtype="<u8").tobytes())
            for a in range(r0, r1, step):
                f.write(self._engine.export_rows(a, min(step, r1 - a)).tobytes())

    @staticmethod
    def load(paths, device: int = 0) -> "ReachabilityMatrix":
        """A matrix from one file or from row-shard files covering [0, n)."""
        from ._engine import DeviceBuild
        if isinstance(paths, (str, bytes)) or hasattr(paths, "__fspath__"):
            paths = [paths]
        heads = []
        for p in paths:
            with open(p, "rb") as f:
                if f.read(8) != ReachabilityMatrix.MAGIC:
                    raise ValueError(f"{p}: not a kano matrix file")
                heads.append((np.frombuffer(f.read(32), dtype="<u8").astype(np.int64), p))
        n = int(heads[0][0][0])
        heads.sort(key=lambda h: int(h[0][1]))
        pos = 0
        for h, p in heads:
            hn, r0, r1, nb = (int(x) for x in h)
            if hn != n or nb != (n + 7) >> 3 or r0 != pos or r1 < r0:
                raise ValueError(f"{p}: shard [{r0}, {r1}) of n={hn} does not continue at {pos}")
            pos = r1
        if pos != n:
            raise ValueError(f"shards cover [0, {pos}) of {n} rows")
        m = ReachabilityMatrix.__new__(ReachabilityMatrix)
        m.container_size = n
        m._engine = DeviceBuild.empty(n, device=device)
        m._containers = None
        m._policies = None
        m._ncontainers = n
        m._lists = None
        nb = (n + 7) >> 3
        for h, p in heads:
            r0, r1 = int(h[1]), int(h[2])
            step = max(1, (64 << 20) // max(nb, 1))
            with open(p, "rb") as f:
                f.seek(40)
                for a in range(r0, r1, step):
                    k = min(step, r1 - a)
                    buf = np.frombuffer(f.read(k * nb), dtype=np.uint8)
                    if buf.size != k * nb:
                        raise ValueError(f"{p}: truncated")
                    m._engine.import_rows(a, buf.reshape(k, nb))
        return m


def _fit(b: BitArray, n: int) -> np.ndarray:
    bits = np.zeros(n, bool)
    src = b.tobool()
    bits[: min(n, src.shape[0])] = src[:n]
    return bool_to_words(bits)
