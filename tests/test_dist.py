"""The row partition and the exchange step of the N > 1 verification
(kano/shard.py, what bench.py's multi-GPU step runs) at world sizes 2 and 3
on CPU with gloo.  The device half (kano_verify_shard -> gather ->
kano_verify_combine across processes) is tests/test_dist_gpu.py."""
import os
import socket
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, staged, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-verification_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from kano.shard import ShardExchange
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W = 5
    x = ShardExchange(torch, W, world, dist=dist, host_staged=staged, device="cpu")
    x.words.copy_(torch.arange(3 * W, dtype=torch.int64) + 1000 * (rank + 1))
    x.gather()
    want = torch.cat([torch.arange(3 * W, dtype=torch.int64) + 1000 * (r + 1)
                      for r in range(world)])
    ok = bool(torch.equal(x.gathered, want))
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("staged", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_exchange_gathers_in_rank_order(world, staged):
    """ShardExchange.gather: every rank's [OR | cross | NAND] words land in
    its slot of the gathered buffer (rank order = row order), directly or
    staged through host memory (the gloo rehearsal path)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, staged, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def test_row_range_covers():
    from kano.shard import owner_of_row, row_range
    for n in (1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            spans = [row_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            for i in range(n):
                a, b = spans[owner_of_row(n, world, i)]
                assert a <= i < b
    with pytest.raises(IndexError):
        owner_of_row(10, 2, 10)
