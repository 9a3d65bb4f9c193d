"""World-size-2 gloo test of the event-batch sharding + window merge (CPU).

A stand-in engine (oracle counts in host memory, exported/imported through the
same raw-pointer calls as the HIP engine) checks that sharding covers every
event once and that the reduced window equals the single-process result.
"""

import ctypes
import os
import socket

import numpy as np
import pytest

from oracle import scipp_semantics as ora


class _HostEngine:
    """Oracle-backed stand-in with BinningEngine's export/import interface."""

    dtype = np.dtype('float64')  # output dtype (float32 for BIFROST-like views)

    def __init__(self, n_screen, edges):
        self.n_screen, self.n_toa_bins = n_screen, len(edges) - 1
        self.edges = edges
        self.window = np.zeros(n_screen * self.n_toa_bins, dtype=np.int64)

    def bin(self, pid, toa):
        pix = ora.pixel_index(pid, np.arange(1, self.n_screen + 1))
        h = ora.detector_histogram(np.arange(self.n_screen), self.n_screen, pix, toa, self.edges)
        self.window += h.ravel().astype(np.int64)

    def export_window_u64(self, ptr):
        w = self.window.astype(np.int64)
        ctypes.memmove(ptr, w.ctypes.data, w.nbytes)

    def import_window_u64(self, ptr):
        w = np.zeros(self.window.shape, dtype=np.int64)
        ctypes.memmove(w.ctypes.data, ptr, w.nbytes)
        self.window = w

    def wait_event(self, ev):
        pass

    # OutputReducer interface: u64 [S] current image | [S] cumulative | [4] totals
    cum = None
    lo, hi = 2, 7  # TOA bin range of the images

    def finalize_partials(self, ptr):
        if self.cum is None:
            self.cum = np.zeros_like(self.window, dtype=np.int64)
        w = self.window.astype(np.int64).reshape(self.n_screen, self.n_toa_bins)
        self.cum += w.ravel()
        c = self.cum.reshape(self.n_screen, self.n_toa_bins)
        out = np.concatenate([w[:, self.lo:self.hi].sum(1), c[:, self.lo:self.hi].sum(1),
                              [w.sum(), w[:, self.lo:self.hi].sum(), c.sum(),
                               c[:, self.lo:self.hi].sum()]]).astype(np.int64)
        ctypes.memmove(ptr, out.ctypes.data, out.nbytes)
        self.window[:] = 0

    def synchronize(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from esslivedata_amd.distributed import WindowReducer, shard_bounds

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(5)
        n = 100_003
        pid = rng.integers(0, 70, n).astype(np.int32)
        toa = rng.integers(-10, 110, n).astype(np.int32)
        edges = np.linspace(0, 100, 11)
        eng = _HostEngine(64, edges)
        lo, hi = shard_bounds(n, rank, world)
        eng.bin(pid[lo:hi], toa[lo:hi])
        # a bin beyond 2^32 on every rank: the int64 reduce stays exact
        eng.window[5] += 3 * 2**32
        red = WindowReducer(eng, torch.device('cpu'))
        root = red.reduce()
        if root:
            full = _HostEngine(64, edges)
            full.bin(pid, toa)
            full.window[5] += world * 3 * 2**32
            q.put(bool(np.array_equal(eng.window, full.window)) and int(eng.window.sum()) > 0)
        else:
            q.put(not eng.window.any())  # this rank's counts moved to the root
    finally:
        dist.destroy_process_group()


def _worker_outputs(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from esslivedata_amd.distributed import OutputReducer, shard_bounds

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        edges = np.linspace(0, 100, 11)
        eng = _HostEngine(64, edges)
        full = _HostEngine(64, edges)
        red = OutputReducer(eng, torch.device('cpu'))
        ok = True
        for batch in range(3):  # cumulative outputs across finalizes
            rng = np.random.default_rng(10 + batch)
            n = 50_001 + batch
            pid = rng.integers(0, 70, n).astype(np.int32)
            toa = rng.integers(-10, 110, n).astype(np.int32)
            lo, hi = shard_bounds(n, rank, world)
            if batch != 1 or rank == 0:  # batch 1: rank 1 gets no events at all
                eng.bin(pid[lo:hi], toa[lo:hi])
                if batch == 1:
                    eng.bin(pid[hi:], toa[hi:])
            res = red.finalize()
            full.bin(pid, toa)
            buf = np.zeros(2 * 64 + 4, dtype=np.int64)
            full.finalize_partials(buf.ctypes.data)
            if rank == 0:
                cur, cum, tot = res
                ok &= np.array_equal(cur, buf[:64].astype(np.float64))
                ok &= np.array_equal(cum, buf[64:128].astype(np.float64))
                ok &= tot == [int(x) for x in buf[128:]] and tot[0] > 0
            else:
                ok &= res is None
        q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_output_reducer_matches_single_process():
    """Sharded binning + reduce of partial outputs == one process over all events."""
    import torch.multiprocessing as mp

    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_outputs, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(results)


def test_shard_bounds_cover_all_events():
    from esslivedata_amd.distributed import shard_bounds

    for n in (0, 1, 7, 1000, 10**9 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def test_gloo_world2_window_reduce_is_exact():
    import torch.multiprocessing as mp

    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True and q.get(timeout=5) is True


def test_assign_banks_loki_dream():
    from esslivedata_amd.distributed import assign_banks

    # LOKI's 9 banks: pixel-id ranges of config/instruments/loki/streams.py:17-27
    ranges = [(1, 802816), (802817, 1032192), (1032193, 1204224), (1204225, 1433600),
              (1433601, 1605632), (1605633, 2007040), (2007041, 2465792), (2465793, 2752512),
              (2752513, 3211264)]
    loki = {f'loki_detector_{i}': b - a + 1 for i, (a, b) in enumerate(ranges)}
    for world in (1, 2, 4, 8):
        a = assign_banks(loki, world)
        assert set(a) == set(loki) and set(a.values()) <= set(range(world))
        load = [sum(loki[b] for b, d in a.items() if d == k) for k in range(world)]
        # LPT bound: no device above max(largest bank, mean + largest bank)
        assert max(load) <= max(max(loki.values()), sum(loki.values()) / world + max(loki.values()))
        if world >= len(loki):
            assert len(set(a.values())) == len(loki)
    assert assign_banks(loki, 3) == assign_banks(dict(reversed(list(loki.items()))), 3)
    with pytest.raises(ValueError):
        assign_banks(loki, 0)


def _worker_subgroup(rank, world, port, q):
    """Ranks 1 and 2 form a subgroup whose root is global rank 2:
    the reducers treat ``dst`` as a global rank; rank 0 stays out."""
    import torch
    import torch.distributed as dist

    from esslivedata_amd.distributed import OutputReducer, WindowReducer

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        grp = dist.new_group([1, 2])
        if rank == 0:
            q.put((rank, True))
            return
        edges = np.linspace(0, 100, 11)
        rng = np.random.default_rng(3)
        n = 40_000
        pid = rng.integers(0, 70, n).astype(np.int32)
        toa = rng.integers(-10, 110, n).astype(np.int32)
        half = n // 2
        eng = _HostEngine(64, edges)
        sl = slice(0, half) if rank == 1 else slice(half, n)
        eng.bin(pid[sl], toa[sl])
        full = _HostEngine(64, edges)
        full.bin(pid, toa)
        ok = True
        # outputs: the root (global rank 2) gets the merged outputs
        red = OutputReducer(eng, torch.device('cpu'), dst=2, group=grp)
        res = red.finalize()
        buf = np.zeros(2 * 64 + 4, dtype=np.int64)
        full.finalize_partials(buf.ctypes.data)
        if rank == 2:
            cur, cum, tot = res
            ok &= np.array_equal(cur, buf[:64].astype(np.float64))
            ok &= tot == [int(x) for x in buf[128:]] and tot[0] > 0
        else:
            ok &= res is None
        # window: the next window merged onto global rank 2
        eng.bin(pid[sl], toa[sl])
        wr = WindowReducer(eng, torch.device('cpu'), dst=2, group=grp)
        root = wr.reduce()
        ok &= root == (rank == 2)
        if rank == 2:
            w2 = _HostEngine(64, edges)
            w2.bin(pid, toa)
            ok &= np.array_equal(eng.window, w2.window) and wr.had_data
            eng.window[:] = 0  # the root's finalize empties its window
        # a window no rank filled: the root's window stays empty, had_data False
        root = wr.reduce(had_data=False)
        if rank == 2:
            ok &= wr.had_data is False and not eng.window.any()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_reducers_subgroup_root_is_global_rank():
    import torch.multiprocessing as mp

    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_subgroup, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert results == {0: True, 1: True, 2: True}


def test_reducers_refuse_float32_engines():
    """Integer merges at finalize are not the reference's per-push float32
    sums beyond 2^24 counts per bin: float32 engines need PushReducer."""
    from esslivedata_amd.distributed import OutputReducer, PushReducer, WindowReducer

    eng = _HostEngine(4, np.linspace(0, 1, 3))
    eng.dtype = np.dtype('float32')
    for cls in (OutputReducer, WindowReducer):
        with pytest.raises(ValueError, match='per push'):
            cls(eng, 'cpu')
    eng.dtype = np.dtype('float64')
    with pytest.raises(ValueError, match='float32 views'):
        PushReducer(eng, 'cpu')
