"""Workflow-protocol parity on the GPU: the drop-in detector-view and monitor
workflows against the oracle's workflow restatement and the reference KATs."""

import json
from pathlib import Path

import numpy as np
import pytest

from oracle import scipp_semantics as ora

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / 'golden'


@pytest.fixture(scope='module', autouse=True)
def _gpu(engine_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def _ts(s):
    from esslivedata_amd.preprocessors import Timestamp

    return Timestamp.from_seconds(s)


def test_detector_service_kat_through_staging_and_workflow():
    """detector_data_test.py:57-131 driven through EventStaging + workflow:
    2000 -> 2000/2000; +3000 -> 5000/3000; +1000 +1000 -> 7000/2000."""
    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.preprocessors import DetectorEvents, EventStaging
    from esslivedata_amd.workflows import GpuDetectorViewWorkflow

    kat = {k['name']: k for k in json.loads((GOLDEN / 'reference_kats.json').read_text())}[
        'detector_service_cumulative_current'
    ]
    inst = synthetic.dummy_panel()
    view = projection.logical_lut(inst.detector_number, dims=('y', 'x'))
    wf = GpuDetectorViewWorkflow('panel_0', view)
    wf.build()
    pre = EventStaging(inst.detector_number)
    rng = np.random.default_rng(1234)
    t = 0
    for sizes, cum, cur in zip(kat['batches'], kat['expected_cumulative'], kat['expected_current']):
        for n in sizes:
            t += 1
            toa = rng.uniform(0, 70_000_000, n).astype(np.int32)
            pid = rng.integers(1, 128**2 + 1, n, dtype=np.int32)
            pre.add(_ts(t), DetectorEvents(pixel_id=pid, time_of_arrival=toa, unit='ns'))
            wf.accumulate({'panel_0': pre.get()}, start_time=_ts(t), end_time=_ts(t + 1))
            pre.release_buffers()
        out = wf.finalize()
        assert out['cumulative'].nansum().value == cum
        assert out['current'].nansum().value == cur
        assert out['counts_total'].value == cur
        assert out['counts_total_cumulative'].value == cum
        assert out['current'].dims == ('y', 'x') and out['current'].dtype == np.float64
        assert 'start_time' in out['current'].coords and 'time' in out['counts_total'].coords
        assert 'start_time' not in out['cumulative'].coords
    with pytest.raises(ValueError):
        wf.finalize()  # empty window: "No data has been added"


def test_geometric_workflow_matches_oracle_with_replicas_range_and_reset():
    from esslivedata_amd import synthetic
    from esslivedata_amd.edges import TOAEdges
    from esslivedata_amd.workflows import (
        DetectorViewParams,
        GeometricViewConfig,
        GpuDetectorViewFactory,
    )

    inst = synthetic.dream_mantle()
    params = DetectorViewParams(
        toa_edges=TOAEdges(start=0.5, stop=71.43, num_bins=100, scale='log'),
        toa_range=(10.0, 40.0),
        pixel_weighting=True,
    )
    factory = GpuDetectorViewFactory(
        detector_numbers={'mantle_detector': inst.detector_number},
        view_config=GeometricViewConfig('cylinder_mantle_z', {'arc_length': 80, 'z': 320}),
        projected_coords={'mantle_detector': inst.coords},
    )
    wf = factory.make_workflow('mantle_detector', params, {})
    wf.build(context_keys={'mantle_detector/transform': 'detector_transform'})
    edges_ms = params.toa_edges.get_edges()
    sl = ora.label_slice(edges_ms, 10.0, 40.0)
    oedges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=np.stack([ora.geometric_screen_index(inst.coords, oedges, k) for k in range(5)]),
        screen_shape=(80, 320),
        toa_edges_ns=ora.to_ns(edges_ms, 'ms'),
        toa_slice=sl,
    )
    geom = ['A', 'A', 'A', 'B', 'B', 'B', 'B']
    for b, g in enumerate(geom):
        pid, toa = synthetic.dream_events(300_000, inst, seed=b)
        wf.accumulate(
            {'mantle_detector': (pid, toa), 'detector_transform': g},
            start_time=_ts(b),
            end_time=_ts(b + 1),
        )
        o.accumulate(pid, toa, geometry=g)
        if b in (1, 4, 6):
            out = wf.finalize()
            exp = o.finalize()
            with np.errstate(divide='ignore', invalid='ignore'):
                w = wf.view.pixel_weights
                np.testing.assert_array_equal(out['current'].values, exp['current'] / w)
                np.testing.assert_array_equal(out['cumulative'].values, exp['cumulative'] / w)
            assert out['counts_in_toa_range'].value == exp['counts_in_toa_range']
            assert out['counts_total_cumulative'].value == exp['counts_total_cumulative']


def test_monitor_workflow_kats_and_range():
    from esslivedata_amd.edges import TOAEdges
    from esslivedata_amd.preprocessors import EventStaging, MonitorEvents
    from esslivedata_amd.workflows import create_gpu_monitor_workflow

    edges = TOAEdges(start=0.0, stop=10.0, num_bins=5, unit='ns')
    wf = create_gpu_monitor_workflow('monitor_1', edges, range_filter=(2.0, 8.0))
    wf.build()
    pre = EventStaging()
    pre.add(_ts(1), MonitorEvents([1, 2, 3, 4, 5], unit='ns'))
    wf.accumulate({'monitor_1': pre.get()}, start_time=_ts(1), end_time=_ts(2))
    pre.release_buffers()
    out = wf.finalize()
    np.testing.assert_array_equal(out['current'].values, [1, 2, 2, 0, 0])
    assert out['counts_total'].value == 5
    assert out['counts_in_toa_range'].value == 4  # bins [2,4),[4,6),[6,8)
    # cumulative 10 vs current 5 over two batches (monitor_workflow_test.py:484-516)
    pre.add(_ts(2), MonitorEvents([1, 2, 3, 4, 5], unit='ns'))
    wf.accumulate({'monitor_1': pre.get()}, start_time=_ts(2), end_time=_ts(3))
    out = wf.finalize()
    assert out['counts_total_cumulative'].value == 10 and out['counts_total'].value == 5
    assert out['current'].coords['time_of_arrival'].unit == 'ns'


def test_monitor_workflow_ms_edges_match_oracle():
    from esslivedata_amd import synthetic
    from esslivedata_amd.edges import TOAEdges
    from esslivedata_amd.workflows import GpuMonitorWorkflow

    edges = TOAEdges()
    wf = GpuMonitorWorkflow('monitor_2', edges, range_filter=(5.0, 30.0))
    o = ora.OracleMonitor(
        toa_edges_ns=edges.edges_ns(),
        range_slice=ora.label_slice(edges.edges_ns() * 1e-6, 5.0, 30.0),
    )
    for b in range(4):
        _, toa = synthetic.fake_detector_events(100_000, 1, 2, seed=b)
        wf.accumulate({'monitor_2': (None, toa)}, start_time=_ts(b), end_time=_ts(b + 1))
        o.accumulate(toa)
    out, exp = wf.finalize(), o.finalize()
    np.testing.assert_array_equal(out['current'].values, exp['current'])
    np.testing.assert_array_equal(out['cumulative'].values, exp['cumulative'])
    assert out['counts_in_toa_range'].value == exp['counts_in_toa_range']


def test_golden_regression_vector_on_gpu():
    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    g = np.load(GOLDEN / 'dream_small.npz')
    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    for strategy in ('atomic', 'partition', 'paged'):
        eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut,
                            pid_offset=view.pid_offset, n_screen=view.n_screen, strategy=strategy)
        eng.stage(g['pid'], g['toa'])
        eng.accumulate(int(g['replica']))
        h = eng.read_histogram().ravel()
        nz = np.nonzero(h)[0]
        np.testing.assert_array_equal(nz, g['hist_index'])
        np.testing.assert_array_equal(h[nz], g['hist_value'])


def test_group_spectra_engine_overlapping_large_and_empty_groups():
    """lde_group_spectra vs numpy group sums of the engine's own histograms:
    overlapping groups, groups larger than one work item, empty groups, both
    selectors, a folded (u64) window and the cumulative pending fold."""
    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    rng = np.random.default_rng(11)
    groups = [rng.choice(view.n_screen, k, replace=False) for k in (1, 63, 64, 65, 700, 25600)]
    groups.insert(2, np.zeros(0, np.int32))
    groups.append(groups[3][:10])  # overlaps another group
    for strategy in ('atomic', 'split'):
        eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut,
                            pid_offset=view.pid_offset, n_screen=view.n_screen, strategy=strategy)
        eng.set_groups(0, groups)
        eng.set_groups(3, [np.arange(view.n_screen)])
        for b in range(3):
            pid, toa = synthetic.dream_events(400_000, inst, seed=20 + b)
            eng.stage(pid, toa)
            eng.accumulate(b % 5)
            cur, cum = eng.read_histogram('current'), eng.read_histogram('cumulative')
            for which, h in (('current', cur), ('cumulative', cum)):
                got = eng.group_spectra(0, which)
                exp = np.asarray([h[g].sum(axis=0) for g in groups])
                np.testing.assert_array_equal(got, exp)
                np.testing.assert_array_equal(eng.group_spectra(3, which)[0], h.sum(axis=0))
            if b == 1:
                eng.finalize()
        eng.set_groups(0, [])  # cleared slot -> empty result
        assert eng.group_spectra(0, 'current').shape == (0, 100)
        with pytest.raises(ValueError):
            eng.set_groups(1, [np.array([view.n_screen])])  # out of range
        eng.close()


def test_geometric_workflow_roi_spectra_match_oracle():
    """roi_spectra_current/cumulative (roi.py:188-266) for rectangles (label and
    index bounds) and polygons on the DREAM view, across finalizes and an ROI
    update, against the oracle on the oracle's histograms."""
    from esslivedata_amd import roi, synthetic
    from esslivedata_amd.edges import TOAEdges
    from esslivedata_amd.workflows import DetectorViewParams, GeometricViewConfig, GpuDetectorViewFactory

    inst = synthetic.dream_mantle()
    params = DetectorViewParams(toa_edges=TOAEdges(start=0.5, stop=71.43, num_bins=100, scale='log'))
    factory = GpuDetectorViewFactory(
        detector_numbers={'mantle_detector': inst.detector_number},
        view_config=GeometricViewConfig('cylinder_mantle_z', {'arc_length': 80, 'z': 320}),
        projected_coords={'mantle_detector': inst.coords},
    )
    aux = {'roi_rectangle': 'job1/roi_rectangle', 'roi_polygon': 'job1/roi_polygon'}
    wf = factory.make_workflow('mantle_detector', params, aux)
    view = wf.view
    ye, xe = view.screen_edges['arc_length'], view.screen_edges['z']
    yc, xc = view.screen_coords['arc_length'], view.screen_coords['z']
    ylo, yhi, xlo, xhi = ye[0], ye[-1], xe[0], xe[-1]
    rects = {0: roi.RectangleROI(x=roi.Interval(xlo + 0.1 * (xhi - xlo), xlo + 0.6 * (xhi - xlo), 'm'),
                                 y=roi.Interval(ylo + 0.2 * (yhi - ylo), ylo + 0.9 * (yhi - ylo), 'm')),
             5: roi.RectangleROI(x=roi.Interval(xlo, xlo + 0.3 * (xhi - xlo), 'm'),
                                 y=roi.Interval(ylo - 1.0, ylo + 0.4 * (yhi - ylo), 'm'))}
    polys = {2: roi.PolygonROI(x=[xlo, xhi, 0.5 * (xlo + xhi)], y=[ylo, ylo, yhi], x_unit='m', y_unit='m')}
    oedges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=np.stack([ora.geometric_screen_index(inst.coords, oedges, k) for k in range(5)]),
        screen_shape=(80, 320), toa_edges_ns=params.toa_edges.edges_ns(),
    )

    def expected(h, rr, pp):
        o_r = [((r.y.min, r.y.max, r.y.unit), (r.x.min, r.x.max, r.x.unit)) for r in rr.values()]
        o_p = [ora.polygon_inside(p.x, p.y, xc, yc) for p in pp.values()]
        return ora.roi_spectra(h.reshape(80, 320, -1), o_r, o_p, oedges['arc_length'], oedges['z'])

    t = 0
    for phase in range(3):
        data = {}
        if phase == 0:
            data = {aux['roi_rectangle']: roi.to_concatenated(rects, 'rectangle'),
                    aux['roi_polygon']: roi.to_concatenated(polys, 'polygon')}
        if phase == 2:  # ROI update: index-based rectangles replace the physical ones
            rects = {1: roi.RectangleROI(x=roi.Interval(10, 250), y=roi.Interval(0, 40)),
                     4: roi.RectangleROI(x=roi.Interval(0, 320), y=roi.Interval(79, 200))}
            data = {aux['roi_rectangle']: roi.to_concatenated(rects, 'rectangle')}
        for b in range(2):
            pid, toa = synthetic.dream_events(300_000, inst, seed=100 + t)
            wf.accumulate({'mantle_detector': (pid, toa), **(data if b == 0 else {})},
                          start_time=_ts(t), end_time=_ts(t + 1))
            o.accumulate(pid, toa)
            t += 1
        out, exp = wf.finalize(), o.finalize()
        ids = list(rects) + list(polys)
        cur, cum = out['roi_spectra_current'], out['roi_spectra_cumulative']
        assert cur.dims == ('roi', 'time_of_arrival') and list(cur.coords['roi'].values) == ids
        np.testing.assert_array_equal(cur.values, expected(exp['histogram_current'], rects, polys))
        np.testing.assert_array_equal(cum.values, expected(exp['histogram_cumulative'], rects, polys))
        assert 'start_time' in cur.coords and 'start_time' not in cum.coords
        assert roi.from_concatenated(out['roi_rectangle']) == rects
        assert roi.from_concatenated(out['roi_polygon']) == polys


def test_bifrost_spectrum_view_float32_matches_oracle():
    """BIFROST unified view: f32 outputs and spectrum_view (bifrost/specs.py:311-349)
    from the cumulative histogram; ROI readbacks of a logical view carry no units."""
    from esslivedata_amd import synthetic
    from esslivedata_amd.workflows import GpuDetectorViewFactory, LogicalViewConfig

    inst = synthetic.bifrost_unified()
    cfg = LogicalViewConfig(transform=lambda a, _s: synthetic.bifrost_transform(a),
                            output_dims=('arc/tube', 'channel/pixel'),
                            spectrum_view=synthetic.bifrost_spectrum_config(10))
    factory = GpuDetectorViewFactory(detector_numbers={'unified_detector': inst.detector_number},
                                     view_config=cfg, out_dtype='float32')
    wf = factory.make_workflow('unified_detector', None, {})
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)[0][None, :],
        screen_shape=(15, 900), toa_edges_ns=inst.edges.edges_ns(), dtype=np.float32,
    )
    for b in range(25):
        pid, toa = synthetic.uniform_events(45_000, 1, 13_500, seed=300 + b)
        wf.accumulate({'unified_detector': (pid, toa)}, start_time=_ts(b), end_time=_ts(b + 1))
        o.accumulate(pid, toa)
        if b % 10 == 9 or b == 24:
            out, exp = wf.finalize(), o.finalize()
            sv = out['spectrum_view']
            assert sv.dims == ('arc', 'detector_number', 'time_of_arrival')
            assert sv.values.dtype == np.float32 and sv.shape == (5, 270, 100)
            np.testing.assert_array_equal(
                sv.values, ora.bifrost_spectrum_view(exp['histogram_cumulative'].reshape(15, 900, -1)
                                                     .astype(np.float64), 10))
            assert out['roi_spectra_current'].shape == (0, 100)
            assert out['roi_rectangle'].coords['x'].unit is None


def test_monitor_workflow_histogram_mode_rebin():
    """Histogram-mode monitors (monitor_workflow.py:101-108) through
    lde_rebin_f64: the reference KATs (monitor_workflow_test.py:190-216,
    518-548), then random histograms in another unit vs the oracle rebin."""
    from esslivedata_amd.dataarray import DataArray, Variable
    from esslivedata_amd.edges import TOAEdges
    from esslivedata_amd.workflows import GpuMonitorWorkflow

    def hist(edges, values, dim='tof', unit='ns'):
        return DataArray(np.asarray(values, dtype=np.float64), (dim,), 'counts',
                         {dim: Variable((dim,), np.asarray(edges, dtype=np.float64), unit)})

    edges = TOAEdges(start=0.0, stop=10.0, num_bins=5, unit='ns')
    wf = GpuMonitorWorkflow('monitor_1', edges)
    wf.build()
    vals = [1.0, 2.0, 3.0, 4.0, 5.0, 4.0, 3.0, 2.0, 1.0, 0.0]
    wf.accumulate({'monitor_1': hist(np.linspace(0, 10, 11), vals)}, start_time=_ts(0),
                  end_time=_ts(1000))
    out = wf.finalize()
    np.testing.assert_array_equal(out['current'].values, [3.0, 7.0, 9.0, 5.0, 1.0])
    assert out['current'].dims == ('time_of_arrival',)
    wf.accumulate({'monitor_1': hist(np.linspace(0, 10, 11), [1.0] * 10, 'time_of_arrival')},
                  start_time=_ts(1000), end_time=_ts(2000))
    out = wf.finalize()
    assert out['current'].sum().value == 10.0 and out['counts_total'].value == 10.0
    assert out['counts_in_toa_range'].value == 10.0
    assert out['cumulative'].sum().value == 35.0
    with pytest.raises(ValueError):
        wf.finalize()

    # ms target edges, ns input histograms with ragged random edges
    edges = TOAEdges()  # 0..71.43 ms, 100 bins
    wf = GpuMonitorWorkflow('monitor_2', edges, range_filter=(5.0, 30.0))
    rng = np.random.default_rng(4)
    e = edges.get_edges()
    cum = np.zeros(len(e) - 1)
    for _ in range(3):
        src = np.sort(rng.uniform(-5e6, 80e6, 3001))
        v = rng.uniform(0, 100, 3000)
        exp = ora.rebin(src * 1e-6, v, e)
        wf.accumulate({'monitor_2': hist(src, v)}, start_time=_ts(0), end_time=_ts(1))
        cum += exp
        out = wf.finalize()
        np.testing.assert_allclose(out['current'].values, exp, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(out['cumulative'].values, cum, rtol=1e-12, atol=1e-9)


def test_roi_spectra_follow_a_detector_move():
    """after a detector move the ROI masks are recomputed on the
    moved projection (the reference's roi.py:31-125 providers depend on the
    rebuilt ScreenMetadata), so physical-unit rectangles and polygons select
    the moved screen cells."""
    from esslivedata_amd import geometry, roi, synthetic
    from esslivedata_amd.workflows import GeometricViewConfig, GpuDetectorViewFactory

    inst = synthetic.loki_bank0(n_replicas=1)
    off = inst.positions - [0.0, 0.0, 5.0]
    res = inst.resolution
    fac = GpuDetectorViewFactory(
        detector_numbers={'loki': inst.detector_number},
        view_config=GeometricViewConfig('xy_plane', res),
        positions={'loki': off}, transforms={'loki': np.array([0.0, 0.0, 5.0])})
    aux = {'roi_rectangle': 'j/roi_rectangle', 'roi_polygon': 'j/roi_polygon'}
    wf = fac.make_workflow('loki', None, aux)
    rects = {0: roi.RectangleROI(x=roi.Interval(-0.2, 0.3, 'm'), y=roi.Interval(-0.4, 0.1, 'm')),
             3: roi.RectangleROI(x=roi.Interval(-0.6, -0.1, 'm'), y=roi.Interval(0.0, 0.5, 'm'))}
    polys = {1: roi.PolygonROI(x=[-0.5, 0.4, 0.0], y=[-0.5, -0.3, 0.45], x_unit='m', y_unit='m')}
    t0 = np.eye(4)
    t0[2, 3] = 5.0
    t1 = t0.copy()
    t1[0, 3] = 0.35  # shifted in x: the screen edges and the ROI cells move
    t1[1, 3] = -0.1
    edges = inst.edges.edges_ns()
    pid, toa = synthetic.uniform_events(1_000_000, 1, 802816, seed=21)
    for step, tr in enumerate([t0, t1, t1]):
        data = {'loki': (pid, toa), 'detector_transform': tr}
        if step == 0:
            data[aux['roi_rectangle']] = roi.to_concatenated(rects, 'rectangle')
            data[aux['roi_polygon']] = roi.to_concatenated(polys, 'polygon')
        wf.accumulate(data, start_time=_ts(step), end_time=_ts(step + 1))
        out = wf.finalize()
        pos = geometry.apply_transform(tr, off)
        coords = geometry.make_xy_plane_coords(pos)
        oedges = {d: ora.screen_edges(coords[d], r) for d, r in res.items()}
        ps = ora.geometric_screen_index(coords, oedges, 0)
        h = ora.detector_histogram(ps, 144 * 144, ora.pixel_index(pid, inst.detector_number),
                                   toa, edges).reshape(144, 144, -1)
        yc = 0.5 * (oedges['y'][1:] + oedges['y'][:-1])
        xc = 0.5 * (oedges['x'][1:] + oedges['x'][:-1])
        o_r = [((r.y.min, r.y.max, r.y.unit), (r.x.min, r.x.max, r.x.unit)) for r in rects.values()]
        o_p = [ora.polygon_inside(p.x, p.y, xc, yc) for p in polys.values()]
        exp = ora.roi_spectra(h, o_r, o_p, oedges['y'], oedges['x'])
        np.testing.assert_array_equal(out['roi_spectra_current'].values, exp)
        assert exp[0].sum() > 0 and exp[2].sum() > 0
    # a rejected move (shape change cannot happen here; an invalid transform
    # raising inside the projection) leaves the placement untouched
    assert np.array_equal(wf._geometry_src.transform, t1)


def test_output_buffers_fresh_without_reuse():
    """``reuse_output_buffers=False`` hands out fresh images each
    finalize (no reliance on reference counts); with reuse, a held image keeps
    its block.  Both exact."""
    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.dummy_panel()
    view = projection.logical_lut(inst.detector_number)
    edges = inst.edges.edges_ns()
    for reuse in (True, False):
        eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                            n_screen=view.n_screen, reuse_output_buffers=reuse)
        held = []
        for k in range(4):
            pid, toa = synthetic.fake_detector_events(50_000, 1, 16384, seed=k)
            eng.stage(pid, toa)
            eng.accumulate(0)
            res = eng.finalize(images=True)
            exp = ora.detector_histogram(view.lut[0], view.n_screen,
                                         ora.pixel_index(pid, inst.detector_number), toa, edges).sum(-1)
            np.testing.assert_array_equal(res.current_image, exp)
            held.append((res.current_image, exp.copy()))
        for img, exp in held:  # earlier results were not overwritten
            np.testing.assert_array_equal(img, exp)
        if not reuse:
            assert len({id(i) for i, _ in held}) == 4
        eng.close()


@pytest.mark.parametrize('num_bins', [100, 1000])
def test_finalize_overlapped_with_next_batch(num_bins):
    """``finalize(wait=False)`` (lde_finalize_begin/_end): the next batch is
    enqueued before the outputs are read; every window's images, totals and
    cumulative match the synchronous engine's, a second pending finalize is
    refused, and a window with no data is refused as with lde_finalize."""
    import torch

    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.with_toa_edges(synthetic.dream_mantle(), num_bins=num_bins, scale='log')
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    kw = dict(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset, n_screen=view.n_screen,
              reuse_output_buffers=False)
    a, b = BinningEngine(**kw), BinningEngine(**kw)
    batches = [synthetic.dream_events(2_000_000, inst, seed=90 + k) for k in range(4)]
    dev = [(torch.as_tensor(p, device='cuda'), torch.as_tensor(t, device='cuda')) for p, t in batches]
    pending, got, exp = None, [], []
    for k, (p, t) in enumerate(dev):
        a.stage_tensors_batch([(p, t)])
        a.accumulate(k % view.n_replicas)
        if pending is not None:
            got.append(pending.result())
        pending = a.finalize(images=True, wait=False)
        if k == 0:
            with pytest.raises(RuntimeError, match='pending'):
                a.finalize(images=True, wait=False)  # one pending finalize per engine
        b.stage_tensors_batch([(p, t)])
        b.accumulate(k % view.n_replicas)
        exp.append(b.finalize(images=True))
    got.append(pending.result())
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g.current_image, e.current_image)
        np.testing.assert_array_equal(g.cumulative_image, e.cumulative_image)
        assert (g.current_total, g.current_in_range, g.cumulative_total, g.cumulative_in_range) == (
            e.current_total, e.current_in_range, e.cumulative_total, e.cumulative_in_range)
    np.testing.assert_array_equal(a.read_histogram('cumulative'), b.read_histogram('cumulative'))
    with pytest.raises(ValueError):
        a.finalize(images=True, wait=False)  # nothing accumulated since
    a.close()
    b.close()


def test_pending_finalize_dropped_or_engine_closed():
    """A pending finalize dropped unread completes itself (the next one is
    accepted); closing the engine completes one that is still held, whose
    outputs stay readable after the close."""
    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.dummy_panel()
    view = projection.logical_lut(inst.detector_number)
    edges = inst.edges.edges_ns()
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, reuse_output_buffers=False)
    pid, toa = synthetic.fake_detector_events(100_000, 1, 16384, seed=3)
    exp = ora.detector_histogram(view.lut[0], view.n_screen, ora.pixel_index(pid, inst.detector_number),
                                 toa, edges).sum(-1)
    eng.stage(pid, toa)
    eng.accumulate(0)
    eng.finalize(images=True, wait=False)  # dropped at once
    eng.stage(pid, toa)
    eng.accumulate(0)
    p = eng.finalize(images=True, wait=False)
    np.testing.assert_array_equal(p.result().current_image, exp)
    eng.stage(pid, toa)
    eng.accumulate(0)
    held = eng.finalize(images=True, wait=False)
    eng.close()
    np.testing.assert_array_equal(held.result().current_image, exp)
