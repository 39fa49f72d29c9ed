"""World-size-2/3 tests of the row partition and its one exchange step
(kano/shard.py) on CPU with the gloo backend: the bench's all-gather of
[or | cross | nand] words combined by OR, and the byte-flag MAX all-reduce.  The
per-shard partials come from the oracle's matrix, so this checks that the
decomposition itself reproduces kano_py's column checks exactly."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _partials(M, gid, r0, r1, n):
    """Shard-local column OR / NAND / cross of rows [r0, r1) as words."""
    from kano._bits import bool_to_words, words_to_bool
    rows = np.array([words_to_bool(M[i], n) for i in range(r0, r1)]).reshape(r1 - r0, n)
    col_or = rows.any(axis=0)
    col_nand = (~rows).any(axis=0)
    cross = np.zeros(n, bool)
    for k, i in enumerate(range(r0, r1)):
        cross |= rows[k] & (gid != gid[i])
    return bool_to_words(col_or), bool_to_words(cross), bool_to_words(col_nand)


def _worker(rank, world, port, name, q, mode="bytes"):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from _golden import cluster
    from kano import shard
    from oracle import kano_oracle as orc
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = cluster(name)
    ref = orc.run_c(obj, label=obj["label"])
    n = ref["n"]
    gid = orc.group_ids_json(obj, obj["label"])
    r0, r1 = shard.row_range(n, world, rank)
    parts = _partials(ref["M"], gid, r0, r1, n)
    if mode == "bytes":
        flags = torch.from_numpy(shard.pack_flags(*parts, n))
        dist.all_reduce(flags, op=dist.ReduceOp.MAX)
        got = shard.decode_flags(flags.numpy(), n)
    else:   # the bench's exchange: all-gather of the words, OR on the receiver
        W = (n + 63) // 64
        words = torch.from_numpy(np.concatenate(parts).astype(np.uint64).view(np.int64))
        assert words.numel() == 3 * W
        gathered = torch.zeros(world * 3 * W, dtype=torch.int64)
        dist.all_gather_into_tensor(gathered, words)
        got = shard.combine_words(gathered.numpy().view(np.uint64), n)
    ok = (got["all_isolated"].tolist() == ref["all_isolated"] and
          got["all_reachable"].tolist() == ref["all_reachable"] and
          got["user_crosscheck"].tolist() == ref["user_crosscheck"])
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("mode", ["words", "bytes"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["s_sparse_500", "q_dirs", "s_broad_300"])
def test_row_partition_gloo(world, name, mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def test_row_range_covers():
    from kano.shard import owner_of_row, row_range
    for n in (0, 1, 7, 100):
        for world in (1, 2, 3, 8):
            spans = [row_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            for i in range(n):
                a, b = spans[owner_of_row(n, world, i)]
                assert a <= i < b
