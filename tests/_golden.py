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
