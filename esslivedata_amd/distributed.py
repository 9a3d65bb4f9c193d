"""Multi-GPU event-batch sharding (no reference counterpart: the reference
has no GPU or collective code).

One process per GPU.  Every rank bins its own share of the event batches into
its own histograms.  Two merge modes, both bit-identical to a single GPU that
binned every event (integer sums are order-independent):

* ``OutputReducer`` (default): every rank keeps its own window and cumulative;
  at each finalize only the outputs the detector view publishes are summed
  onto the root -- uint64 partial images (current, cumulative) and totals,
  2*S + 4 words (400 KB for DREAM) instead of the 10 MB window -- with one
  ``torch.distributed.reduce`` (backend ``nccl`` = RCCL over xGMI on ROCm).
* ``WindowReducer``: sums the windows onto the root as uint64 (exact in every
  window state, also after a rank's u32 window folded into u64), which then
  finalizes as a single GPU would; needed when the full (S, T) histogram is
  published.
* ``PushReducer`` (float32 views, BIFROST): the reference adds every push to
  float32 accumulators (SRC/preprocessors/accumulators.py:129-135, the cast of
  config/instruments/bifrost/specs.py:295), which rounds once per push beyond
  2^24 counts per bin; merging at finalize would round once in total.  So the
  ranks' exact counts of each push are summed onto the root before that
  push's f32 add: one reduce of S*T uint64 per push.  The two reducers above
  refuse float32 engines.

``dst``/``root`` is always a global rank (``torch.distributed`` collectives
take global ranks for ``dst`` in any group).

Pixel-range (bank) sharding needs no collective: see :func:`assign_banks`.

With the ``gloo`` backend (CPU tests, or ranks sharing one GPU) the device
buffers travel through host copies, since gloo reduces host tensors.
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


def assign_banks(bank_sizes: dict[str, int], world: int) -> dict[str, int]:
    """Pixel-range sharding (SURVEY 8(e) axis 2): each detector bank is its own
    job/workflow (e.g. LOKI's 9 banks, config/instruments/loki/streams.py:17-27;
    DREAM's 5, dream/streams.py:17-23), so banks are placed on devices whole and
    need no collective.  Greedy longest-processing-time placement by expected
    load (pixels, or events/s if known): largest bank first onto the least
    loaded device; ties broken by device index, so the result is deterministic.
    Returns ``{bank: device}``."""
    if world < 1:
        raise ValueError('world must be >= 1')
    load = [0] * world
    out: dict[str, int] = {}
    for name, size in sorted(bank_sizes.items(), key=lambda kv: (-int(kv[1]), kv[0])):
        if int(size) < 0:
            raise ValueError(f'bank {name!r} has negative size')
        d = min(range(world), key=lambda i: (load[i], i))
        out[name] = d
        load[d] += int(size)
    return out


class _Reducer:
    """Reduce of one device buffer onto ``dst`` with stream ordering against
    the engine: the engine's stream waits for the previous reduce before it
    rewrites the buffer (RCCL runs the collective asynchronously)."""

    def __init__(self, engine, buf, *, dst: int, group) -> None:
        import torch.distributed as dist

        self.engine = engine
        self.buf = buf
        self.dst = dst
        self.group = group
        self._host = buf.is_cuda and dist.get_backend(group) == 'gloo'
        self._after = None  # event recorded after the last reduce

    def _before_write(self) -> None:
        if self._after is not None:
            self.engine.wait_event(self._after)
            self._after = None

    def _order_after_engine(self) -> None:
        """The collective (on torch's current stream) after the engine's
        writes of the buffer: a stream wait, no host synchronization (when the
        engine runs on torch's current stream the two are in order already)."""
        import torch

        if not self.buf.is_cuda:
            self.engine.synchronize()
            return
        cur = torch.cuda.current_stream(self.buf.device)
        sp = self.engine.stream_ptr
        if sp == cur.cuda_stream:
            return
        es = torch.cuda.ExternalStream(sp, device=self.buf.device)
        ev = torch.cuda.Event()
        ev.record(es)
        cur.wait_event(ev)

    def _reduce(self) -> bool:
        import torch.distributed as dist

        self._order_after_engine()
        root = dist.get_rank() == self.dst  # dst is a global rank
        if self._host:
            hb = self.buf.cpu()
            dist.reduce(hb, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group)
            if root:
                self.buf.copy_(hb)
        else:
            dist.reduce(self.buf, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group)
        self._mark()
        return root

    def _mark(self) -> None:
        """Record the point after torch's last use of the buffer."""
        if self.buf.is_cuda:
            import torch

            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.buf.device))
            self._after = ev


class OutputReducer(_Reducer):
    _hbuf = None  # page-locked host copy of the reduced outputs (root)

    def _to_host(self):
        """The reduced buffer on the host: one async copy into a reused
        page-locked tensor on the collective's stream, then a stream sync
        (``Tensor.cpu()`` would allocate pageable memory every finalize)."""
        import torch

        if not self.buf.is_cuda:
            return self.buf.numpy()
        if self._hbuf is None:
            self._hbuf = torch.empty(self.buf.shape, dtype=self.buf.dtype, pin_memory=True)
        self._hbuf.copy_(self.buf, non_blocking=True)
        torch.cuda.current_stream(self.buf.device).synchronize()
        return self._hbuf.numpy()

    """Sums every rank's finalize outputs onto the root (see module doc)."""

    def __init__(self, engine, device, *, dst: int = 0, group=None) -> None:
        import torch

        _refuse_f32(engine, 'OutputReducer')
        self.S = engine.n_screen
        # [S] current image | [S] cumulative image | [4] totals | [1] windows
        # that held data (summed: the merged window is empty only if all were)
        super().__init__(engine, torch.zeros(2 * self.S + 5, dtype=torch.int64, device=device),
                         dst=dst, group=group)
        self.had_data = True  # root: any rank's window held data at the last finalize

    def finalize(self, had_data: bool = True):
        """Collective.  On the root: (current image, cumulative image, totals)
        as float64 numpy arrays and a list of 4 ints; elsewhere None.  ``had_data``: this rank accumulated since
        its last finalize (merged into ``self.had_data`` on the root)."""
        self._before_write()
        self.engine.finalize_partials(self.buf.data_ptr())
        self._order_after_engine()
        self.buf[2 * self.S + 4].fill_(1 if had_data else 0)
        if not self._reduce():
            return None
        h = self._to_host()
        S = self.S
        dt = self.engine.dtype
        self.had_data = bool(h[2 * S + 4])
        return h[:S].astype(dt), h[S : 2 * S].astype(dt), [int(x) for x in h[2 * S : 2 * S + 4]]


class WindowReducer(_Reducer):
    """Sums every rank's window into the root's window (uint64 SUM: exact for
    any count and after a rank's u32 window has folded into u64)."""

    def __init__(self, engine, device, *, dst: int = 0, group=None) -> None:
        import torch

        _refuse_f32(engine, 'WindowReducer')
        self.n = engine.n_screen * engine.n_toa_bins
        # [S*T] window | [1] ranks whose window held data
        super().__init__(engine, torch.zeros(self.n + 1, dtype=torch.int64, device=device),
                         dst=dst, group=group)
        self.had_data = True  # root: any rank's window held data at the last reduce

    def reduce(self, had_data: bool = True) -> bool:
        """Collective; returns True on the root, which now holds the merged
        window; the other ranks' windows are emptied (their counts moved).
        ``had_data``: this rank accumulated since its last finalize.  When no
        rank had data the root's window is left empty (``self.had_data`` is
        False), so its finalize raises 'No data has been added' as a single
        workflow's would."""
        self._before_write()
        self.engine.export_window_u64(self.buf.data_ptr())
        self._order_after_engine()
        self.buf[self.n].fill_(1 if had_data else 0)
        root = self._reduce()
        if not root:
            self.buf.zero_()  # this rank's counts now live on the root
            self._mark()
        else:
            self.had_data = bool(int(self.buf[self.n].item()))
            if not self.had_data:
                return True  # nothing to import: the window stays empty
        self._before_write()  # the reduced buffer before the engine reads it
        self.engine.import_window_u64(self.buf.data_ptr())
        return root


class PushReducer(_Reducer):
    """Per-push exact merge of a float32 view (see the module doc): every
    rank bins its share of a push with ``accumulate_push`` (exact counts into
    the reduce buffer, its own accumulators untouched), the counts are summed
    onto the root, and the root adds the sum as ONE push (``push_counts``:
    f32 += float32(count)).  Only the root's accumulators hold data; it
    finalizes as a single GPU that binned every push would."""

    def __init__(self, engine, device, *, dst: int = 0, group=None) -> None:
        import torch

        if engine.dtype != 'float32':
            raise ValueError('PushReducer is for float32 views; integer views merge exactly at '
                             'finalize (OutputReducer / WindowReducer)')
        self.n = engine.n_screen * engine.n_toa_bins
        super().__init__(engine, torch.zeros(self.n, dtype=torch.int64, device=device), dst=dst,
                         group=group)

    def push(self, replica: int, has_events: bool = True) -> bool:
        """Collective.  Bins this rank's staged events of the push (zeros when
        ``has_events`` is False and nothing is staged) and merges the push
        onto the root; returns True on the root."""
        self._before_write()
        if has_events:
            self.engine.accumulate_push(int(replica), self.buf.data_ptr())
        else:
            self._order_after_engine()
            self.buf.zero_()
        root = self._reduce()
        if root:
            self._before_write()
            # the next push's export runs behind this add on the engine stream;
            # a push without events zeroes the buffer after waiting for it
            self.engine.push_counts(self.buf.data_ptr())
        return root


def _refuse_f32(engine, what: str) -> None:
    if engine.dtype == 'float32':
        raise ValueError(f'{what} merges integer counts at finalize, which is not the '
                         "reference's per-push float32 sum beyond 2^24 counts per bin: "
                         'float32 views merge per push (PushReducer)')
