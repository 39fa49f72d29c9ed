"""Helpers shared by the parity tests: load golden records / clusters, and the
canonical layouts of tests/golden/make_golden.py."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def expected(name):
    with open(os.path.join(GOLDEN, "expected", name + ".json")) as f:
        return json.load(f)


def cluster(name):
    with open(os.path.join(GOLDEN, "clusters", name + ".json")) as f:
        return json.load(f)


def cluster_names():
    return sorted(f[:-5] for f in os.listdir(os.path.join(GOLDEN, "clusters")))


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rows01_to_words(rows, n):
    W = (n + 63) // 64
    out = np.zeros((len(rows), W), dtype=np.uint64)
    for r, s in enumerate(rows):
        buf = np.zeros(W * 64, dtype=np.uint8)
        buf[:n] = np.frombuffer(s.encode(), np.uint8) - ord("0")
        out[r] = np.packbits(buf, bitorder="little").view("<u8")
    return out


def words_to_rows01(words, n):
    out = []
    for w in np.asarray(words, dtype=np.uint64).reshape(-1, (n + 63) // 64 if n else 1):
        b = np.unpackbits(w.view(np.uint8), bitorder="little")[:n]
        out.append("".join("1" if x else "0" for x in b))
    return out


def csr_sha(off, lst):
    off = np.ascontiguousarray(off, dtype=np.int64)
    lst = np.ascontiguousarray(lst, dtype=np.int32)
    return hashlib.sha256(off.tobytes() + lst.tobytes()).hexdigest()


def lists_to_csr(lists):
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    if lists:
        off[1:] = np.cumsum([len(l) for l in lists])
    flat = np.array([x for l in lists for x in l], dtype=np.int32)
    return off, flat


def index_list_matches(got, exp) -> bool:
    """An index list against make_golden.py's record: the list itself, or
    (long lists of the big configs) count + sha256 of the int32 array."""
    got = np.ascontiguousarray(np.asarray(got, dtype=np.int32))
    if isinstance(exp, dict):
        return got.shape[0] == exp["count"] and sha(got) == exp["sha256"]
    return got.tolist() == exp


_MIX = (np.uint64(0x9e3779b97f4a7c15), np.uint64(0xbf58476d1ce4e5b9),
        np.uint64(0x94d049bb133111eb), np.uint64(0xD6E8FEB86659FD93))


def row_digest(words) -> np.ndarray:
    """Host form of kano_rows_digest: per row, sum over k of
    mix64(row[k] ^ k * 0xD6E8FEB86659FD93) mod 2^64 (splitmix64 finaliser)."""
    w = np.atleast_2d(np.asarray(words, dtype=np.uint64))
    k = np.arange(w.shape[1], dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = w ^ (k * _MIX[3])
        z = z + _MIX[0]
        z = (z ^ (z >> np.uint64(30))) * _MIX[1]
        z = (z ^ (z >> np.uint64(27))) * _MIX[2]
        z = z ^ (z >> np.uint64(31))
        return z.sum(axis=1, dtype=np.uint64)


def container_lists_csr(cls, sel_off, sel_pol):
    """Container.select_policies for every pod as one CSR (pod-major) from
    the engine's class-level lists (kano_get_classes / kano_get_select_csr)."""
    cls = np.asarray(cls, dtype=np.int64)
    cnt = np.diff(sel_off)[cls]
    off = np.zeros(cls.shape[0] + 1, dtype=np.int64)
    np.cumsum(cnt, out=off[1:])
    starts = np.repeat(sel_off[:-1][cls], cnt)
    pos = np.arange(off[-1], dtype=np.int64) - np.repeat(off[:-1], cnt)
    return off, np.asarray(sel_pol, dtype=np.int32)[starts + pos]


def allow_lists_csr(n, alw_off, alw_pods):
    """Container.allow_policies for every pod (ascending policy ids) from the
    engine's per-policy allowed-pod lists (kano_get_allow_csr)."""
    P = alw_off.shape[0] - 1
    pol = np.repeat(np.arange(P, dtype=np.int32), np.diff(alw_off))
    order = np.lexsort((pol, alw_pods))
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(alw_pods, minlength=n), out=off[1:])
    return off, pol[order]
