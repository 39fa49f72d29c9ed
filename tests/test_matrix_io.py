"""The matrix row format: M's rows as kano_py holds
them, bitarray bytes in big-endian bit order (kano_py/kano/model.py:136-139,
bitarray.tobytes()), exported from / imported into HBM by libkano_hip.so, and
the row-shard file format built on it (kano/model.py ReachabilityMatrix.save /
load).  Pinned by kano_py's golden matrices."""
import os

import numpy as np
import pytest

from _golden import cluster, expected

pytestmark = pytest.mark.gpu

IO_CLUSTERS = ["q_dirs", "q_types", "s_sparse_50", "s_sparse_200", "s_broad_300"]


def _golden_rows_bytes(name, n):
    rows = expected(name)["M"]
    bits = np.array([[c == "1" for c in r] for r in rows], dtype=bool).reshape(n, n)
    return np.packbits(bits, axis=1, bitorder="big")   # bitarray(row).tobytes()


def _build(name):
    from kano import model
    from kano.synth import objects_from_json
    cs, ps = objects_from_json(cluster(name), model)
    return model.ReachabilityMatrix.build_matrix(cs, ps)


def _names():
    out = []
    for nm in IO_CLUSTERS:
        try:
            if "M" in expected(nm):
                out.append(nm)
        except FileNotFoundError:
            pass
    return out


@pytest.mark.parametrize("name", _names())
def test_row_bytes_match_kano_py(name):
    m = _build(name)
    n = m.container_size
    assert np.array_equal(m.row_bytes(), _golden_rows_bytes(name, n))


def test_save_load_roundtrip_and_shards(tmp_path):
    from kano import algorithm as alg
    from kano.model import ReachabilityMatrix
    m = _build("s_sparse_500")
    n = m.container_size
    ref = m.engine.rows(0, n)
    p = tmp_path / "m.kano"
    m.save(str(p))
    assert os.path.getsize(p) == 40 + n * ((n + 7) // 8)
    back = ReachabilityMatrix.load(str(p))
    assert np.array_equal(back.engine.rows(0, n), ref)
    assert alg.all_isolated(back) == alg.all_isolated(m)
    # row shards written separately, loaded in any order
    cut = 123
    m.save(str(tmp_path / "a.kano"), rows=(0, cut))
    m.save(str(tmp_path / "b.kano"), rows=(cut, n))
    both = ReachabilityMatrix.load([str(tmp_path / "b.kano"), str(tmp_path / "a.kano")])
    assert np.array_equal(both.engine.rows(0, n), ref)
    with pytest.raises(ValueError):
        ReachabilityMatrix.load([str(tmp_path / "b.kano")])
    bad = tmp_path / "bad.kano"
    bad.write_bytes(b"NOTKANO!" + bytes(32))
    with pytest.raises(ValueError):
        ReachabilityMatrix.load(str(bad))


def test_import_clears_pad_bits():
    from kano._engine import DeviceBuild
    n = 77
    eng = DeviceBuild.empty(n)
    rng = np.random.default_rng(5)
    rows = rng.integers(0, 256, size=(n, (n + 7) // 8), dtype=np.uint8)   # pad bits set too
    eng.import_rows(0, rows)
    back = eng.export_rows(0, n)
    bits = np.unpackbits(rows, axis=1, bitorder="big")[:, :n]
    assert np.array_equal(back, np.packbits(bits, axis=1, bitorder="big"))
    words = eng.rows(0, n)
    lsb = np.packbits(np.pad(bits, ((0, 0), (0, 128 - n))), axis=1, bitorder="little")
    assert np.array_equal(words, lsb.view("<u8"))
    eng.close()
