"""Row-sharded verification across ranks: one process per GPU (SURVEY.md
§8(e)); what bench.py's N > 1 step runs.

Rows of M (source pods) are independent: M[i] = OR_{p in S(i)} allow_p
(kano_py/kano/model.py:158-160), so rank r builds rows row_range(n, N, r)
with no communication (kano_verify_shard).  The column checks are
existentials / universals over rows and combine over shards:

  all_isolated[j]    = NOT OR_r colOR_r[j]          (algorithm.py:12-17)
  all_reachable[j]   = NOT OR_r colNAND_r[j]        (algorithm.py:4-9)
  user_crosscheck[j] = OR_r cross_r[j]              (algorithm.py:27-42)

RCCL has no bitwise reduction, so the one exchange is an all-gather of every
rank's [OR | cross | NAND] words (3 W u64 = 3n/8 bytes per rank; 37.5 KB at
100k pods) over xGMI, OR-ed on the device by kano_verify_combine, which also
lists the results.  system_isolation comes from the rank owning the row;
policy_shadow's output is ordered by container, so each rank emits its own
rows' pairs and rank order is the global order.

With the nccl (RCCL) backend the exchange is native by default: the engine
runs the shard's checks, the all-gather and the combine in one call
(kano_verify_gather), issuing ncclAllGather itself on its stream through
torch's communicator (``ProcessGroupNCCL._comm_ptr()``), so no Python or
c10d work sits between the shard's last kernel and the combine
(KANO_NATIVE_EXCHANGE=0 keeps the torch collective).  With the gloo backend
(several ranks rehearsing on one device, or CPU-only collectives) the words
travel through host memory: ``host_staged``.
"""
from __future__ import annotations

import os

from typing import Optional, Tuple


def row_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Rows [r0, r1) of rank ``rank`` of ``world`` (contiguous, balanced)."""
    return rank * n // world, (rank + 1) * n // world


def owner_of_row(n: int, world: int, i: int) -> int:
    """The rank whose row_range holds row i."""
    if not 0 <= i < n:
        raise IndexError(i)
    r = (i * world) // n
    while row_range(n, world, r)[1] <= i:   # floor rounding: at most one step
        r += 1
    while row_range(n, world, r)[0] > i:
        r -= 1
    return r


class ShardExchange:
    """The N > 1 verification step of one rank: kano_verify_shard, the
    all-gather of the ranks' column words, kano_verify_combine.

    ``eng`` is the rank's DeviceBuild (rows = row_range(...)), created on
    ``stream`` (a torch.cuda.Stream) so that the collective is ordered after
    the shard's kernels on the same stream.  ``dist`` None with ``nranks``
    > 1 emulates rank 0 of nranks on one device (other ranks' words zero: a
    timing diagnostic, results are partial)."""

    def __init__(self, torch, W: int, nranks: int, dist=None, stream=None,
                 host_staged: Optional[bool] = None, device: str = "cuda",
                 native: Optional[bool] = None):
        self.torch, self.W, self.nranks, self.dist, self.stream = torch, W, nranks, dist, stream
        if host_staged is None:
            host_staged = dist is not None and dist.get_backend() == "gloo"
        self.host_staged = host_staged
        self.words = torch.zeros(3 * W, dtype=torch.int64, device=device)
        self.gathered = torch.zeros(nranks * 3 * W, dtype=torch.int64, device=device)
        if host_staged:
            self._hw = torch.zeros(3 * W, dtype=torch.int64)
            self._hg = torch.zeros(nranks * 3 * W, dtype=torch.int64)
        self.comm = None   # ncclComm_t of the native exchange
        if native is None:
            native = (dist is not None and not host_staged
                      and os.environ.get("KANO_NATIVE_EXCHANGE", "1") != "0")
        if native:
            self.comm = self._rccl_comm()
        # emulated rank 0 through the engine's own gather call (comm NULL);
        # KANO_EMUL_NATIVE=0 keeps the shard / torch copy / combine form
        self.emulate_native = (dist is None and nranks > 1
                               and os.environ.get("KANO_EMUL_NATIVE", "1") != "0")
        self.mode = ("emulated" if dist is None else "rccl-native" if self.comm
                     else "host-staged" if host_staged else "torch-collective")

    def _rccl_comm(self) -> Optional[int]:
        """torch's RCCL communicator for this device (created by one
        all-gather, as the first collective on the device does)."""
        torch, dist = self.torch, self.dist
        try:
            if dist.get_backend() != "nccl" or dist.get_world_size() != self.nranks:
                return None
            ctx = torch.cuda.stream(self.stream) if self.stream is not None else None
            if ctx is not None:
                with ctx:
                    dist.all_gather_into_tensor(self.gathered, self.words)
            else:
                dist.all_gather_into_tensor(self.gathered, self.words)
            torch.cuda.synchronize()
            pg = dist.distributed_c10d._get_default_group()
            be = pg._get_backend(torch.device("cuda", torch.cuda.current_device()))
            ptr = int(be._comm_ptr())
            return ptr or None
        except Exception:   # noqa: BLE001 (no raw communicator: the torch collective)
            return None

    def gather(self) -> None:
        """Every rank's words into ``gathered`` (rank order)."""
        torch, dist = self.torch, self.dist
        if dist is None:
            # (the engine writes the words and reads the gathered buffer on its
            # own streams when it has them: order the copy through the device)
            on_dev = self.stream is None and self.words.is_cuda
            if on_dev:
                torch.cuda.synchronize()
            self.gathered[:3 * self.W].copy_(self.words)
            if on_dev:
                torch.cuda.synchronize()
        elif self.host_staged:
            if self.words.is_cuda:
                torch.cuda.synchronize()      # the shard's kernels wrote the words
            self._hw.copy_(self.words)
            dist.all_gather_into_tensor(self._hg, self._hw)
            self.gathered.copy_(self._hg)
            if self.gathered.is_cuda:
                torch.cuda.synchronize()
        else:
            # (the engine's kernels and the collective are on different streams
            # when the engine has its own: order them through the device)
            on_dev = self.stream is None and self.words.is_cuda
            if on_dev:
                torch.cuda.synchronize()
            dist.all_gather_into_tensor(self.gathered, self.words)
            if on_dev:
                torch.cuda.synchronize()

    def _run(self, eng, gid, sys_row, shadow, count_only, pairs, idx):
        if self.dist is None and self.nranks > 1 and self.emulate_native:
            # emulated rank 0 (a timing diagnostic): one engine call like the
            # native exchange, the all-gather a device copy (comm NULL)
            return eng.verify_gather(0, self.nranks, gid=gid, sys_row=sys_row, shadow=shadow,
                                     shadow_count_only=count_only, pairs=pairs, idx=idx)
        if self.comm:
            return eng.verify_gather(self.comm, self.nranks, gid=gid, sys_row=sys_row,
                                     shadow=shadow, shadow_count_only=count_only, pairs=pairs,
                                     idx=idx)
        eng.verify_shard(self.words.data_ptr(), gid=gid, sys_row=sys_row, shadow=shadow,
                         shadow_count_only=count_only)
        self.gather()
        return eng.verify_combine(self.gathered.data_ptr(), self.nranks, pairs=pairs, idx=idx,
                                  shadow_count_only=count_only)

    def verify(self, eng, gid="stored", sys_row: int = 0, shadow: bool = True,
               count_only: bool = False, pairs=None, idx=None) -> dict:
        """kano_py's checks for this rank (algorithm.py:4-80): the column
        lists are global, system_isolation is None unless this rank owns
        sys_row, the shadow pairs are this rank's rows' part."""
        if self.stream is None or self.comm or (self.dist is None and self.emulate_native):
            # (the native exchange issues everything on the engine's own
            # stream: no torch stream context needed, a few us less host time
            # per step)
            return self._run(eng, gid, sys_row, shadow, count_only, pairs, idx)
        with self.torch.cuda.stream(self.stream):
            return self._run(eng, gid, sys_row, shadow, count_only, pairs, idx)

    def checks(self, eng, gid="stored", sys_row: int = 0, idx=None) -> dict:
        """The same exchange over the rows as they stand after incremental
        updates (kano_checks_shard; kano_verify would rebuild from the
        tables): global column lists, the owner's system_isolation."""
        def run():
            eng.checks_shard(self.words.data_ptr(), gid=gid, sys_row=sys_row)
            self.gather()
            return eng.verify_combine(self.gathered.data_ptr(), self.nranks, idx=idx)
        if self.stream is None:
            return run()
        with self.torch.cuda.stream(self.stream):
            return run()
