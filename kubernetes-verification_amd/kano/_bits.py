"""A bitarray-compatible bit vector for the drop-in API.

The reference returns ``bitarray.bitarray`` objects (default endian "big")
from ``getrow``/``getcol`` and stores them in ``Policy.working_select_set`` /
``working_allow_set`` (kano_py/kano/model.py:119-121,177-184).  The GPU box's
Python has no ``bitarray`` package, so the drop-in ships this subset: same
indexing (ints 0/1), ``count``, ``setall``, ``&``/``|``/``^``/``~``, in-place
forms, ``any``/``all``/``index``/``search``, ``to01``/``tolist``/``tobytes``
(big-endian bit order inside each byte, pad bits zero) and equality with real
bitarrays through ``to01()``.

Storage is the engine's layout: little-endian uint64 words, bit j in word
j >> 6 at position j & 63 (include/kano_hip.h).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import numpy as np

_U64 = np.uint64


def _nwords(n: int) -> int:
    return (n + 63) >> 6


def _tail_mask(n: int) -> Optional[np.uint64]:
    r = n & 63
    return None if r == 0 else _U64((1 << r) - 1)


def words_to_bool(words: np.ndarray, n: int) -> np.ndarray:
    b = np.unpackbits(np.ascontiguousarray(words, dtype="<u8").view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def bool_to_words(bits: np.ndarray) -> np.ndarray:
    n = bits.shape[0]
    nw = _nwords(n)
    buf = np.zeros(nw * 64, dtype=np.uint8)
    buf[:n] = bits.astype(np.uint8)
    return np.packbits(buf, bitorder="little").view("<u8").astype(_U64)


def set_bit_indices(words: np.ndarray, n: int) -> np.ndarray:
    """Ascending indices j < n whose bit is set."""
    return np.flatnonzero(words_to_bool(words, n))


class BitArray:
    """Packed bit vector with the bitarray API subset the reference uses."""

    __slots__ = ("_wd", "_n")

    def __init__(self, init=None, endian: str = "big"):
        if endian != "big":
            raise ValueError("only the reference's default endianness ('big') is supported")
        if init is None:
            self._n, self._wd = 0, np.zeros(0, _U64)
        elif isinstance(init, (int, np.integer)):
            if init < 0:
                raise ValueError("cannot create bitarray with negative length")
            # bitarray(n) is uninitialised in the reference (quirk Q10); zeros here
            self._n, self._wd = int(init), np.zeros(_nwords(int(init)), _U64)
        elif isinstance(init, str):
            s = init.replace("_", "").replace(" ", "")
            if any(ch not in "01" for ch in s):
                raise ValueError("bitarray string may only contain '0' and '1'")
            self._n = len(s)
            self._wd = bool_to_words(np.frombuffer(s.encode(), np.uint8) == ord("1"))
        elif isinstance(init, BitArray):
            self._n, self._wd = len(init), init._words().copy()
        elif hasattr(init, "to01"):
            b = BitArray(init.to01())
            self._n, self._wd = b._n, b._wd
        else:
            bits = np.asarray([1 if x else 0 for x in init], dtype=bool)
            self._n, self._wd = bits.shape[0], bool_to_words(bits)

    # -- construction helpers ------------------------------------------
    @classmethod
    def from_words(cls, words: np.ndarray, n: int) -> "BitArray":
        obj = cls.__new__(cls)
        w = np.array(words, dtype=_U64, copy=True).reshape(-1)[: _nwords(n)]
        m = _tail_mask(n)
        if m is not None and w.size:
            w[-1] &= m
        obj._wd, obj._n = w, n
        return obj

    def _words(self) -> np.ndarray:
        return self._wd

    def _store(self, words: np.ndarray) -> None:
        self._wd = words

    def words(self) -> np.ndarray:
        """Copy of the packed LSB-first uint64 words."""
        return self._words().copy()

    # -- sequence protocol ---------------------------------------------
    def __len__(self) -> int:
        return self._n

    def _norm(self, i: int) -> int:
        i = int(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError("bitarray index out of range")
        return i

    def __getitem__(self, key):
        if isinstance(key, slice):
            idx = range(*key.indices(self._n))
            bits = self.tobool()[list(idx)] if len(idx) else np.zeros(0, bool)
            return BitArray.from_words(bool_to_words(bits), len(idx))
        i = self._norm(key)
        return int((int(self._words()[i >> 6]) >> (i & 63)) & 1)

    def __setitem__(self, key, value):
        if isinstance(key, slice):
            idx = list(range(*key.indices(self._n)))
            bits = self.tobool()
            if isinstance(value, (int, bool, np.integer)):
                bits[idx] = bool(value)
            else:
                vals = list(value) if not hasattr(value, "tolist") else value.tolist()
                if len(vals) != len(idx):
                    raise ValueError("slice assignment length mismatch")
                bits[idx] = np.asarray(vals, dtype=bool)
            self._store(bool_to_words(bits))
            return
        i = self._norm(key)
        w = self._words().copy()
        bit = _U64(1 << (i & 63))
        w[i >> 6] = (w[i >> 6] | bit) if value else (w[i >> 6] & ~bit)
        self._store(w)

    def __iter__(self):
        return iter(self.tolist())

    # -- queries --------------------------------------------------------
    def tobool(self) -> np.ndarray:
        return words_to_bool(self._words(), self._n)

    def count(self, value=1, *args) -> int:
        if args:
            return int(self[slice(*args)].count(value))
        ones = int(np.unpackbits(self._words().view(np.uint8)).sum()) if self._n else 0
        return ones if value else self._n - ones

    def any(self) -> bool:
        return bool(self._words().any())

    def all(self) -> bool:
        return self.count(0) == 0

    def index(self, value=1, *args) -> int:
        hits = np.flatnonzero(self.tobool() == bool(value))
        if args:
            lo = args[0]
            hi = args[1] if len(args) > 1 else self._n
            hits = hits[(hits >= lo) & (hits < hi)]
        if hits.size == 0:
            raise ValueError(f"{int(bool(value))} not in bitarray")
        return int(hits[0])

    def search(self, sub, limit=None) -> List[int]:
        pat = BitArray(sub).tolist() if not isinstance(sub, BitArray) else sub.tolist()
        bits = self.tolist()
        out, m = [], len(pat)
        for s in range(0, self._n - m + 1):
            if bits[s:s + m] == pat:
                out.append(s)
                if limit is not None and len(out) >= limit:
                    break
        return out

    def setall(self, value) -> None:
        w = np.full(_nwords(self._n), ~_U64(0) if value else _U64(0), dtype=_U64)
        m = _tail_mask(self._n)
        if m is not None and w.size:
            w[-1] &= m
        self._store(w)

    def to01(self) -> str:
        return self.tobool().astype(np.uint8).tobytes().translate(bytes.maketrans(b"\x00\x01", b"01")).decode()

    def tolist(self) -> List[int]:
        return self.tobool().astype(np.uint8).tolist()

    def tobytes(self) -> bytes:
        return np.packbits(self.tobool().astype(np.uint8), bitorder="big").tobytes()

    def endian(self) -> str:
        return "big"

    def copy(self) -> "BitArray":
        return BitArray.from_words(self._words(), self._n)

    # -- bitwise --------------------------------------------------------
    def _other_words(self, other) -> np.ndarray:
        if isinstance(other, BitArray):
            if len(other) != self._n:
                raise ValueError("bitarrays of equal length expected for bitwise operation")
            return other._words()
        if hasattr(other, "to01"):
            return self._other_words(BitArray(other.to01()))
        return NotImplemented

    def _binop(self, other, op):
        ow = self._other_words(other)
        if ow is NotImplemented:
            return NotImplemented
        return BitArray.from_words(op(self._words(), ow), self._n)

    def __and__(self, o):
        return self._binop(o, np.bitwise_and)

    def __or__(self, o):
        return self._binop(o, np.bitwise_or)

    def __xor__(self, o):
        return self._binop(o, np.bitwise_xor)

    def __iand__(self, o):
        r = self.__and__(o)
        self._store(r._wd)
        return self

    def __ior__(self, o):
        r = self.__or__(o)
        self._store(r._wd)
        return self

    def __ixor__(self, o):
        r = self.__xor__(o)
        self._store(r._wd)
        return self

    def __invert__(self):
        return BitArray.from_words(~self._words(), self._n)

    # -- comparison / display ------------------------------------------
    def __eq__(self, other):
        if isinstance(other, BitArray):
            return self._n == len(other) and bool(np.array_equal(self._words(), other._words()))
        if hasattr(other, "to01"):
            return self.to01() == other.to01()
        return NotImplemented

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    __hash__ = None

    def __repr__(self) -> str:
        return f"bitarray('{self.to01()}')" if self._n else "bitarray()"

    __str__ = __repr__


def bitarray_from_indices(n: int, idx: Iterable[int]) -> BitArray:
    bits = np.zeros(n, bool)
    bits[np.asarray(list(idx), dtype=np.int64)] = True
    return BitArray.from_words(bool_to_words(bits), n)
