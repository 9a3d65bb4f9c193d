"""Event-batch sharding on the real engine (the reducers had only
run against a host stand-in).

Two spawned ranks share cuda:0 and talk gloo (the reducers stage the device
buffers through host copies for gloo), each binning its own shard with a real
``BinningEngine`` on its own HIP stream.  Checked against one engine (or the C
oracle) that binned every event:

* ``OutputReducer`` over three finalizes, one of which a rank gets no events;
* ``WindowReducer`` after both ranks' u32 windows folded into u64 (> 2^32
  events per window) with one bin beyond 2^32 on each rank -- exact only with
  the uint64 export / reduce / import (lde_export_window_u64).
"""

import os
import socket

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)


def _dream():
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    return inst, view


def _engine(view, edges, **kw):
    from esslivedata_amd.engine import BinningEngine

    return BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                         n_screen=view.n_screen, device=0, toa_range=(10, 90), **kw)


def _outputs_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from esslivedata_amd import synthetic
    from esslivedata_amd.distributed import OutputReducer, shard_bounds

    _init(rank, world, port)
    try:
        inst, view = _dream()
        edges = inst.edges.edges_ns()
        eng = _engine(view, edges)  # engine-owned stream
        full = _engine(view, edges) if rank == 0 else None
        red = OutputReducer(eng, torch.device('cuda', 0))
        ok = True
        for batch in range(3):
            n = 600_001 + batch
            pid, toa = synthetic.dream_events(n, inst, seed=60 + batch)
            lo, hi = shard_bounds(n, rank, world)
            r = batch % view.n_replicas
            if batch == 1:  # rank 1 gets nothing, rank 0 everything
                if rank == 0:
                    eng.stage(pid, toa)
                    eng.accumulate(r)
            else:
                eng.stage(pid[lo:hi], toa[lo:hi])
                eng.accumulate(r)
            res = red.finalize()
            if rank == 0:
                full.stage(pid, toa)
                full.accumulate(r)
                ref = full.finalize(images=True)
                cur, cum, tot = res
                ok &= bool(np.array_equal(cur, ref.current_image))
                ok &= bool(np.array_equal(cum, ref.cumulative_image))
                ok &= tot == [ref.current_total, ref.current_in_range, ref.cumulative_total,
                              ref.cumulative_in_range] and tot[0] > 0
            else:
                ok &= res is None
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _bifrost_worker(rank, world, port, q):
    """float32 view (BIFROST unified detector, 45 bank streams): every rank
    bins its share of each push's bank messages; ``PushReducer`` sums the
    push's exact counts onto the root before the root's float32 add, so the
    root's images equal one engine that binned every message, push by push.
    Then one bin is driven past 2^24 counts: a first push of 2^24 events
    (split over the ranks), then pushes of one event each.  The reference's
    per-push float32 sum stays at 2^24 (16777216 + 1 rounds to even); the
    root's cumulative must equal that, not the exact count rounded once
    (accumulators.py:129-135, bifrost/specs.py:295)."""
    import torch
    import torch.distributed as dist

    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.distributed import PushReducer
    from esslivedata_amd.engine import BinningEngine

    _init(rank, world, port)
    try:
        inst = synthetic.bifrost_unified()
        view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
        edges = inst.edges.edges_ns()

        def make():
            return BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                                 n_screen=view.n_screen, device=0, out_dtype='float32',
                                 toa_range=(5, 95))

        eng = make()
        full = make() if rank == 0 else None
        red = PushReducer(eng, torch.device('cuda', 0))
        ok = True
        for window in range(3):
            for push in range(2):
                for bank in range(45):  # bifrost/streams.py:22-43: one message per bank
                    pid, toa = synthetic.fake_detector_events(
                        1000, 1 + 300 * bank, 300 * (bank + 1), seed=1000 * window + 100 * push + bank)
                    if bank % world == rank:
                        eng.stage(pid, toa)
                    if rank == 0:
                        full.stage(pid, toa)
                red.push(0)
                if rank == 0:
                    full.accumulate(0)
            if rank == 0:
                ref = full.finalize(images=True)
                res = eng.finalize(images=True)
                ok &= res.current_image.dtype == np.float32
                ok &= bool(np.array_equal(res.current_image, ref.current_image))
                ok &= bool(np.array_equal(res.cumulative_image, ref.cumulative_image))
                ok &= [res.current_total, res.cumulative_total] == [ref.current_total,
                                                                    ref.cumulative_total]
                ok &= ref.current_total > 0
        # one bin past 2^24: pid 1, a TOA inside bin 50
        if rank == 0:
            eng.clear()
        t50 = int((edges[50] + edges[51]) / 2)
        dev = torch.device('cuda', 0)
        big = 1 << 24
        share = big // world + (1 if rank < big % world else 0)
        pushes = [share] + [1 if rank == world - 1 else 0 for _ in range(4)]
        exp = np.float32(0)
        for k, n in enumerate(pushes):
            if n:
                eng.stage_tensors(torch.full((n,), 1, dtype=torch.int32, device=dev),
                                  torch.full((n,), t50, dtype=torch.int32, device=dev))
            red.push(0, has_events=n > 0)
            exp = np.float32(exp + np.float32(big if k == 0 else 1))
        if rank == 0:
            res = eng.finalize(hists=True)
            s0 = int(view.lut[0][0])  # pixel 1's screen
            got = res.cumulative_hist[s0, 50]
            ok &= got == exp == np.float32(big)  # per-push rounding, not 2^24 + 4
            ok &= res.cumulative_total == big + 4  # exact integer totals
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


FIREHOSE = 100_000_000
FIRE_MSGS = 44  # 4.4e9 events per rank: the u32 window folds into u64


def _window_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from esslivedata_amd import synthetic
    from esslivedata_amd.distributed import WindowReducer

    _init(rank, world, port)
    try:
        inst, view = _dream()
        edges = inst.edges.edges_ns()
        dev = torch.device('cuda', 0)
        eng = _engine(view, edges)
        pid, toa = synthetic.torch_dream_events(10_000_000, inst, 40 + rank, dev)
        # one pixel, one TOA bin, 4.4e9 times: a bin beyond 2^32 on this rank
        fp = torch.full((FIREHOSE,), int(inst.detector_number[1234]), dtype=torch.int32, device=dev)
        ft = torch.full((FIREHOSE,), 30_000_000, dtype=torch.int32, device=dev)
        eng.stage_tensors_batch([(pid, toa)] + [(fp, ft)] * FIRE_MSGS)
        eng.accumulate(0)
        red = WindowReducer(eng, dev)
        root = red.reduce()
        got = eng.read_histogram('current')
        if root:
            from oracle import c_oracle
            from oracle import scipp_semantics as ora

            ps = ora.geometric_pixel_screen(inst.coords, inst.resolution)
            o = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, edges)
            for r in range(world):
                p2, t2 = synthetic.torch_dream_events(10_000_000, inst, 40 + r, dev)
                o.accumulate(p2.cpu().numpy(), t2.cpu().numpy(), 0)
            exp = o.hist.astype(np.float64).reshape(view.n_screen, -1)
            s = int(ps[0][1234])
            b = int(ora.hist_bin_index(np.array([30_000_000]), edges)[0])
            exp[s, b] += world * FIRE_MSGS * FIREHOSE
            ok = bool(np.array_equal(got, exp)) and got[s, b] > 2.0**33
            res = eng.finalize(images=True)
            ok &= res.current_total == int(exp.sum()) == res.cumulative_total
            q.put((rank, ok))
        else:
            q.put((rank, not got.any()))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _rccl_worker(rank, world, port, q):
    """The RCCL path itself (backend 'nccl' with device_id, device-buffer
    reduces, as bench.py --gpus N runs it), on one rank: the box has one GPU
    and RCCL refuses two ranks on one device.  OutputReducer and WindowReducer
    through RCCL must return exactly what the engine alone finalizes."""
    import torch
    import torch.distributed as dist

    from esslivedata_amd import synthetic
    from esslivedata_amd.distributed import OutputReducer, WindowReducer

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)
    try:
        ok = dist.get_backend() == 'nccl'
        inst, view = _dream()
        edges = inst.edges.edges_ns()
        eng = _engine(view, edges)
        ref = _engine(view, edges)
        red = OutputReducer(eng, dev)
        for batch in range(2):
            pid, toa = synthetic.torch_dream_events(3_000_000, inst, 70 + batch, dev)
            for e in (eng, ref):
                e.stage_tensors_batch([(pid, toa)])
                e.accumulate(batch)
            cur, cum, tot = red.finalize()
            exp = ref.finalize(images=True)
            ok &= bool(np.array_equal(cur, exp.current_image))
            ok &= bool(np.array_equal(cum, exp.cumulative_image))
            ok &= tot == [exp.current_total, exp.current_in_range, exp.cumulative_total,
                          exp.cumulative_in_range] and tot[0] > 0
        pid, toa = synthetic.torch_dream_events(3_000_000, inst, 80, dev)
        for e in (eng, ref):
            e.stage_tensors_batch([(pid, toa)])
            e.accumulate(2)
        ok &= WindowReducer(eng, dev).reduce() is True
        ok &= bool(np.array_equal(eng.read_histogram('current'), ref.read_histogram('current')))
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(target, world=2, timeout=240):
    import torch.multiprocessing as mp

    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=timeout) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert results == {r: True for r in range(world)}, results


@pytest.fixture(scope='module', autouse=True)
def _gpu(engine_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def test_output_reducer_two_ranks_real_engines():
    _run(_outputs_worker)


def test_window_reducer_after_u64_fold_two_ranks():
    _run(_window_worker)


def test_push_reducer_float32_view_two_ranks_past_2_24():
    _run(_bifrost_worker)


def test_rccl_reducers_single_rank():
    _run(_rccl_worker, world=1)
