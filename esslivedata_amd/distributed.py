"""Multi-GPU event-batch sharding with an RCCL window merge (no reference
counterpart: the reference has no GPU or collective code).

One process per GPU.  Every rank bins its own share of the event batches into
its own uint32 window; at each finalize the windows are summed onto the root
with ``torch.distributed.reduce`` (backend ``nccl`` = RCCL over xGMI on ROCm).
Integer sums are order-independent, so the merged counts are bit-identical to
a single-GPU run over all events.  The root then finalizes (cumulative +=
window, images, totals); the other ranks drop their window.
"""

from __future__ import annotations

import os


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous event-batch shard [lo, hi) of rank ``rank``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('invalid rank/world')
    base, rem = divmod(int(n), world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def dist_env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (
        int(os.environ.get('RANK', '0')),
        int(os.environ.get('LOCAL_RANK', '0')),
        int(os.environ.get('WORLD_SIZE', '1')),
    )


class WindowReducer:
    """Sums every rank's window into the root's window (SUM over uint32)."""

    def __init__(self, engine, device, *, dst: int = 0, group=None) -> None:
        import torch

        self.engine = engine
        self.dst = dst
        self.group = group
        n = engine.n_screen * engine.n_toa_bins
        self.buf = torch.zeros(n, dtype=torch.int32, device=device)

    def reduce(self) -> bool:
        """Collective; returns True on the root (which now holds the merged window)."""
        import torch.distributed as dist

        self.engine.export_window(self.buf.data_ptr())
        dist.reduce(self.buf, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group)
        root = dist.get_rank(self.group) == self.dst
        if root:
            self.engine.import_window(self.buf.data_ptr())
        return root
