"""The sharded detector-view workflow on real engines.

Two spawned ranks share cuda:0 and talk gloo (the reducers stage device
buffers through host copies), each running ``ShardedDetectorViewWorkflow``
over its own ``GpuDetectorViewWorkflow`` on its shard of every batch.  Only
rank 0 is handed the context (detector transform, ROI requests); the wrapper
broadcasts it, so a detector move mid-run re-projects and resets the
cumulative on both ranks in the same batch.  The root's outputs are compared
bit-exactly with one workflow that saw every event and every context value
(reference semantics: accumulators.py:116-131, geometry_signal.py:27-51).
Also: a collective ``clear()``, a batch in which one rank has no events, the
window merge with ROI spectra, and bank placement through
``GpuDetectorViewFactory(device=...)`` driven by ``assign_banks``.
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


def _t(ns):
    from esslivedata_amd.preprocessors import Timestamp

    return Timestamp.from_ns(ns)


def _loki_factory(roi: bool):
    from esslivedata_amd import synthetic
    from esslivedata_amd.workflows import GeometricViewConfig, GpuDetectorViewFactory

    inst = synthetic.loki_bank0(n_replicas=3)
    off = inst.positions - [0.0, 0.0, 5.0]
    fac = GpuDetectorViewFactory(
        detector_numbers={'loki': inst.detector_number},
        view_config=GeometricViewConfig('xy_plane', inst.resolution, pixel_noise=inst.pixel_noise),
        positions={'loki': off}, transforms={'loki': np.array([0.0, 0.0, 5.0])})
    return inst, fac


def _transforms():
    t0 = np.eye(4)
    t0[2, 3] = 5.0
    t1 = t0.copy()
    c, s = np.cos(0.3), np.sin(0.3)
    t1[:3, :3] = [[c, 0, s], [0, 1, 0], [-s, 0, c]]
    t1[0, 3] = 0.4
    return t0, t1


def _rois():
    from esslivedata_amd import roi

    rects = {0: roi.RectangleROI(x=roi.Interval(-0.3, 0.2, 'm'), y=roi.Interval(-0.4, 0.3, 'm'))}
    polys = {2: roi.PolygonROI(x=[-0.5, 0.4, 0.0], y=[-0.5, -0.3, 0.45], x_unit='m', y_unit='m')}
    return roi.to_concatenated(rects, 'rectangle'), roi.to_concatenated(polys, 'polygon')


def _same(a, b) -> bool:
    if set(a) != set(b):
        return False
    for k in a:
        va, vb = a[k], b[k]
        if k in ('roi_rectangle', 'roi_polygon'):
            continue  # request readbacks: compared by content elsewhere
        if not np.array_equal(np.asarray(va.values), np.asarray(vb.values)):
            return False
        if va.dims != vb.dims or set(va.coords) != set(vb.coords):
            return False
    return True


def _sharded_worker(rank, world, port, q, merge):
    import torch
    import torch.distributed as dist

    from esslivedata_amd import synthetic
    from esslivedata_amd.distributed import shard_bounds
    from esslivedata_amd.sharded import ShardedDetectorViewWorkflow

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        roi_on = merge == 'window'
        inst, fac = _loki_factory(roi_on)
        aux = {'roi_rectangle': 'j/roi_rectangle', 'roi_polygon': 'j/roi_polygon'}
        local = fac.make_workflow('loki', None, aux)
        if not roi_on:
            local._roi_support = False  # outputs merge: images and totals only
        sw = ShardedDetectorViewWorkflow(local, torch.device('cuda', 0), merge=merge)
        full = None
        if rank == 0:
            full = fac.make_workflow('loki', None, aux)
            if not roi_on:
                full._roi_support = False
        t0, t1 = _transforms()
        rect, poly = _rois()
        # (transform, rank 1 gets events, clear before) per batch
        plan = [(t0, True, False), (t0, False, False), (t1, True, False), (t1, True, True),
                (t1, True, False)]
        ok = True
        for b, (tr, r1_events, clear) in enumerate(plan):
            if clear:
                sw.clear()
                if full is not None:
                    full.clear()
            n = 400_003 + b
            pid, toa = synthetic.uniform_events(n, 1, 802816, seed=70 + b)
            lo, hi = shard_bounds(n, rank, world) if r1_events else ((0, n) if rank == 0 else (0, 0))
            data = {}
            if hi > lo:
                data['loki'] = (pid[lo:hi], toa[lo:hi])
            context = {'detector_transform': tr}
            if b == 0 and roi_on:
                context.update({aux['roi_rectangle']: rect, aux['roi_polygon']: poly})
            if rank == 0:
                data.update(context)
            sw.accumulate(data, start_time=_t(b), end_time=_t(b + 1))
            out = sw.finalize()
            if rank == 0:
                full.accumulate({'loki': (pid, toa), **context}, start_time=_t(b), end_time=_t(b + 1))
                ref = full.finalize()
                why = []
                if not _same(out, ref):
                    why.append('outputs differ from one workflow: ' + ', '.join(
                        k for k in ref if k in out and not np.array_equal(
                            np.asarray(out[k].values), np.asarray(ref[k].values))))
                if not float(ref['counts_total'].values) > 0:
                    why.append('no counts')
                if roi_on and not out['roi_spectra_current'].values.sum() > 0:
                    why.append('empty ROI spectra')
                # the root stamps the window like one workflow: int64 ns scalars
                st, tt = out['current'].coords['start_time'], out['current'].coords['time']
                if (st.value, tt.value, tt.unit, np.asarray(st.values).dtype) != (b, b + 1, 'ns', np.int64) \
                        or 'time' in out['cumulative'].coords:
                    why.append(f'window time coords {st}, {tt}')
                # the move (batch 2) and the clear (batch 3) restart the
                # cumulative: it equals the current image there
                same_cc = bool(np.array_equal(out['cumulative'].values, out['current'].values))
                if same_cc != (b in (0, 2, 3)):
                    why.append('cumulative restart')
                if why:
                    ok = f'batch {b}: ' + '; '.join(why)
                    break
            elif out is not None:
                ok = 'non-root returned outputs'
                break
        q.put((rank, ok))
    except Exception as e:  # pragma: no cover - reported through the queue
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _subgroup_worker(rank, world, port, q):
    """Three ranks; the view is sharded over the subgroup {1, 2} whose root is
    global rank 2: the root's context (a detector move) reaches
    rank 1, and rank 2 publishes outputs equal to one workflow's."""
    import torch
    import torch.distributed as dist

    from esslivedata_amd import synthetic
    from esslivedata_amd.distributed import shard_bounds
    from esslivedata_amd.sharded import ShardedDetectorViewWorkflow

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        grp = dist.new_group([1, 2])
        if rank == 0:
            q.put((rank, True))
            return
        inst, fac = _loki_factory(False)
        local = fac.make_workflow('loki')
        local._roi_support = False
        sw = ShardedDetectorViewWorkflow(local, torch.device('cuda', 0), root=2, group=grp)
        full = None
        if rank == 2:
            full = fac.make_workflow('loki')
            full._roi_support = False
        t0, t1 = _transforms()
        ok = True
        for b, tr in enumerate([t0, t1, t1]):
            n = 300_001 + b
            pid, toa = synthetic.uniform_events(n, 1, 802816, seed=170 + b)
            lo, hi = shard_bounds(n, rank - 1, 2)
            data = {'loki': (pid[lo:hi], toa[lo:hi])}
            if rank == 2:
                data['detector_transform'] = tr
            sw.accumulate(data, start_time=_t(b), end_time=_t(b + 1))
            out = sw.finalize()
            if rank == 2:
                full.accumulate({'loki': (pid, toa), 'detector_transform': tr},
                                start_time=_t(b), end_time=_t(b + 1))
                ref = full.finalize()
                if out is None or not _same(out, ref) or not float(ref['counts_total'].values) > 0:
                    ok = f'batch {b}: root outputs differ'
                    break
            elif out is not None:
                ok = 'non-root returned outputs'
                break
        q.put((rank, ok))
    except Exception as e:  # pragma: no cover - reported through the queue
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _push_worker(rank, world, port, q):
    """merge='push' (float32 views): a BIFROST-like float32 view
    with its spectrum view over batches where the root, the other rank or
    both have no share of the events, one batch without events at all and a
    window in which only the other rank had events; the root's outputs equal
    one workflow's after every finalize."""
    import torch
    import torch.distributed as dist

    from esslivedata_amd import synthetic
    from esslivedata_amd.distributed import shard_bounds
    from esslivedata_amd.sharded import ShardedDetectorViewWorkflow
    from esslivedata_amd.workflows import GpuDetectorViewFactory, LogicalViewConfig

    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        inst = synthetic.bifrost_unified()
        cfg = LogicalViewConfig(transform=lambda a, _s: synthetic.bifrost_transform(a),
                                output_dims=('arc/tube', 'channel/pixel'),
                                spectrum_view=synthetic.bifrost_spectrum_config(10))
        fac = GpuDetectorViewFactory(detector_numbers={'unified_detector': inst.detector_number},
                                     view_config=cfg, out_dtype='float32')
        sw = ShardedDetectorViewWorkflow(fac.make_workflow('unified_detector', None, {}),
                                         torch.device('cuda', 0))
        assert sw._merge == 'push'
        full = fac.make_workflow('unified_detector', None, {}) if rank == 0 else None
        # (ranks with a share of the batch, finalize after it)
        plan = [((0, 1), False), ((1,), True), ((0,), False), ((), False), ((1,), True),
                ((0, 1), True), ((1,), True), ((0, 1), True)]
        ok = True
        for b, (owners, fin) in enumerate(plan):
            n = 45_000 * 14 + b
            pid, toa = synthetic.uniform_events(n, 1, 13_500, seed=500 + b)
            data = {}
            if rank in owners:
                lo, hi = shard_bounds(n, owners.index(rank), len(owners))
                data['unified_detector'] = (pid[lo:hi], toa[lo:hi])
            sw.accumulate(data, start_time=_t(b), end_time=_t(b + 1))
            if rank == 0:
                full.accumulate({'unified_detector': (pid, toa)} if owners else {},
                                start_time=_t(b), end_time=_t(b + 1))
            if not fin:
                continue
            out = sw.finalize()
            if rank == 0:
                ref = full.finalize()
                if out is None or not _same(out, ref):
                    ok = f'batch {b}: root outputs differ from one workflow'
                    break
                if out['current'].values.dtype != np.float32 or not out['current'].values.sum() > 0:
                    ok = f'batch {b}: float32 image expected'
                    break
            elif out is not None:
                ok = 'non-root returned outputs'
                break
        q.put((rank, ok))
    except Exception as e:  # pragma: no cover - reported through the queue
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _outputs_merge(rank, world, port, q):
    _sharded_worker(rank, world, port, q, 'outputs')


def _window_merge(rank, world, port, q):
    _sharded_worker(rank, world, port, q, 'window')


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


def test_sharded_workflow_outputs_merge_with_move_and_clear():
    _run(_outputs_merge)


def test_sharded_workflow_window_merge_with_roi_spectra():
    _run(_window_merge)


def test_sharded_workflow_push_merge_float32_ranks_without_events():
    _run(_push_worker)


def test_sharded_workflow_subgroup_root_is_global_rank():
    _run(_subgroup_worker, world=3)


def test_outputs_merge_refuses_grouped_outputs():
    import torch
    import torch.distributed as dist

    from esslivedata_amd.sharded import ShardedDetectorViewWorkflow

    inst, fac = _loki_factory(True)
    wf = fac.make_workflow('loki')  # geometric views support ROIs
    if not dist.is_initialized():
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()))
        dist.init_process_group('gloo', rank=0, world_size=1)
    try:
        with pytest.raises(ValueError, match='window'):
            ShardedDetectorViewWorkflow(wf, torch.device('cuda', 0), merge='outputs')
    finally:
        dist.destroy_process_group()


def test_bank_placement_through_factory_devices():
    """SURVEY 8(e) axis 2: LOKI-like banks placed whole on devices by
    ``assign_banks`` (no collective), each bank's workflow created on its
    device through ``GpuDetectorViewFactory(device=...)``; every bank's image
    matches the oracle."""
    import torch

    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.distributed import assign_banks
    from esslivedata_amd.workflows import GpuDetectorViewFactory, LogicalViewConfig
    from oracle import scipp_semantics as ora

    n_dev = torch.cuda.device_count()
    sizes = {f'loki_detector_{i}': (9 - i) * 4096 for i in range(9)}
    placement = assign_banks(sizes, n_dev)
    first = 1
    for bank, size in sizes.items():
        dn = np.arange(first, first + size, dtype=np.int32).reshape(-1, 64)
        first += size
        fac = GpuDetectorViewFactory(detector_numbers={bank: dn}, view_config=LogicalViewConfig(),
                                     device=placement[bank])
        wf = fac.make_workflow(bank)
        assert wf.engine.info()['device'] == placement[bank]
        pid, toa = synthetic.uniform_events(50_000, int(dn.min()) - 10, int(dn.max()) + 10, seed=size)
        wf.accumulate({bank: (pid, toa)}, start_time=_t(0), end_time=_t(1))
        out = wf.finalize()
        v = projection.logical_lut(dn)
        exp = ora.detector_histogram(v.lut[0], v.n_screen, ora.pixel_index(pid, dn), toa,
                                     synthetic.TOAEdges().edges_ns()).sum(-1).reshape(dn.shape)
        np.testing.assert_array_equal(out['current'].values, exp)
