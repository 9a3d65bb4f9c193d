"""Wavelength mode on the GPU: the per-event coordinate
pass (lde_coord.hip) + every binning strategy vs the CPU oracle, bit-exact.

The coordinate arithmetic follows include/lde.h ``lde_set_coord_lut`` and is
restated in ``oracle.scipp_semantics.coordinate_lookup``.  The reference's own
interpolation lives in essreduce (absent here), so agreement with the
reference's wavelengths is unpinned; agreement between engine and oracle is
exact, including events whose coordinate sits exactly on an edge.
"""

import numpy as np
import pytest

from oracle import scipp_semantics as ora

pytestmark = pytest.mark.gpu

STRATEGIES = ['atomic', 'partition', 'paged', 'split', 'pixel', 'wide']


@pytest.fixture(scope='module', autouse=True)
def _gpu(engine_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def _t(ns):
    from esslivedata_amd.preprocessors import Timestamp

    return Timestamp.from_ns(ns)


def _dream_setup(table_min=77.5, scale='linear'):
    from esslivedata_amd import projection, synthetic, wavelength
    from esslivedata_amd.edges import WavelengthEdges

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    tab = synthetic.dream_wavelength_table(distance_min=table_min)
    lt = wavelength.pixel_ltotal(inst.positions, source_position=(0, 0, -synthetic.DREAM_L1))
    d = wavelength.distance_per_pid(inst.detector_number, lt, view.pid_offset, view.lut.shape[1])
    edges = WavelengthEdges(start=0.2, stop=3.6, num_bins=100, scale=scale).get_edges()
    return inst, view, tab, lt, d, edges


def _pixel_screen(inst):
    edges = {k: ora.screen_edges(inst.coords[k], r) for k, r in inst.resolution.items()}
    r = next(iter(inst.coords.values())).shape[0]
    return np.stack([ora.geometric_screen_index(inst.coords, edges, k) for k in range(r)])


@pytest.mark.parametrize('scale,table_min', [('linear', 77.5), ('log', 77.75)])
@pytest.mark.parametrize('strategy', STRATEGIES)
def test_dream_wavelength_matches_oracle(strategy, scale, table_min):
    """DREAM mantle, skewed events, three batches cycling replicas; a table
    starting at 77.75 m leaves part of the mantle off the grid (dropped)."""
    from esslivedata_amd import synthetic
    from esslivedata_amd.engine import BinningEngine

    inst, view, tab, lt, d, edges = _dream_setup(table_min, scale)
    lo, hi = 10, 90
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy, toa_range=(lo, hi))
    eng.set_coordinate_lut(d, tab.table, dist0=tab.distance0, dist_step=tab.distance_step,
                           time0=tab.time0, time_step=tab.time_step)
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number, pixel_screen=_pixel_screen(inst),
        screen_shape=(80, 320), toa_edges_ns=edges, toa_slice=(lo, hi),
        coordinate=ora.wavelength_mode(lt, tab.table, tab.distance0, tab.distance_step,
                                       tab.time0, tab.time_step))
    for batch in range(3):
        pid, toa = synthetic.dream_events(1_500_000, inst, seed=200 + batch)
        pid[:1000] = 229376  # unknown ids on both sides of the LUT
        pid[1000:2000] = 720897
        toa[2000:2100] = -5  # before the grid
        eng.stage(pid[:700_000], toa[:700_000])
        eng.stage(pid[700_000:], toa[700_000:])
        eng.accumulate(batch % view.n_replicas)
        o.accumulate(pid, toa)
    res = eng.finalize(hists=True)
    exp = o.finalize()
    # PIXEL needs footprints that fit LDS; the mantle's do not (WIDE runs)
    assert eng.info()['last_strategy'] == (strategy if strategy != 'pixel' else 'wide')
    assert exp['histogram_cumulative'].sum() > 1_000_000  # most events binned
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
    np.testing.assert_array_equal(res.current_image.reshape(80, 320), exp['current'])
    assert res.current_in_range == exp['counts_in_toa_range']
    assert res.cumulative_total == exp['counts_total_cumulative']


# keyed SPLIT pass variant (diagnostics build): the general event pass (bin
# loops, grid coordinate per event) beside the default FAST one
KEYED_VARIANTS = [{'LDE_COORD_FIXED_BIN': '0'},
                  # few sieve blocks over the key stream
                  {'LDE_SPLIT_GRID': '9'}]


@pytest.mark.parametrize('variant', range(len(KEYED_VARIANTS)))
def test_dream_wavelength_keyed_variants(variant, knobs):
    knobs(**KEYED_VARIANTS[variant])
    test_dream_wavelength_matches_oracle('split', 'log', 77.75)


@pytest.mark.parametrize('strategy', STRATEGIES)
def test_coordinates_on_edges_are_half_open(strategy):
    """Grid nodes carry the edge values themselves: an event at a node has
    fx = fy = 0 and its coordinate equals an edge exactly, so it must land in
    the bin that edge opens (the last edge: dropped), as scipp's hist does."""
    from esslivedata_amd import projection
    from esslivedata_amd.engine import BinningEngine

    edges = np.geomspace(0.5, 9.5, 41)
    nd, nt, dt = 6, 20, 4096.0
    tab = np.array([[edges[(i * nt + j) % 41] for j in range(nt)] for i in range(nd)])
    tab[2, 5] = np.nan  # a NaN cell: events next to it are dropped
    dn = np.arange(1, 65, dtype=np.int32)
    view = projection.logical_lut(dn)
    ltot = (np.arange(64) % nd).astype(np.float64) * 0.5 + 3.0  # exact grid distances
    ltot[7] = np.nan
    ltot[9] = 100.0  # off the grid
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy)
    eng.set_coordinate_lut(ltot, tab, dist0=3.0, dist_step=0.5, time0=0.0, time_step=dt)
    rng = np.random.default_rng(11)
    n = 400_000
    pid = rng.integers(1, 65, n).astype(np.int32)
    node = rng.random(n) < 0.5  # half exactly on time nodes, half anywhere
    toa = np.where(node, rng.integers(0, nt, n) * int(dt),
                   rng.integers(-100, int(dt) * nt + 100, n)).astype(np.int32)
    eng.stage(pid, toa)
    eng.accumulate(0)
    res = eng.finalize(hists=True)
    o = ora.OracleDetectorView(dn, np.arange(64)[None], (64,), edges,
                               coordinate=ora.wavelength_mode(ltot, tab, 3.0, 0.5, 0.0, dt))
    o.accumulate(pid, toa)
    exp = o.finalize()
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    # the node events really sit on edges (ties exercised)
    c = ora.wavelength_mode(ltot, tab, 3.0, 0.5, 0.0, dt)(pid - 1, toa)
    assert np.isin(c[node], edges).mean() > 0.6


def test_wavelength_rebind_keeps_counts_and_uses_new_distances():
    """A second ``set_coordinate_lut`` (detector moved: new Ltotal) keeps the
    binned counts; later events use the new distances."""
    from esslivedata_amd import synthetic
    from esslivedata_amd.engine import BinningEngine

    inst, view, tab, lt, d, edges = _dream_setup()
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy='auto')
    kw = dict(dist0=tab.distance0, dist_step=tab.distance_step, time0=tab.time0,
              time_step=tab.time_step)
    eng.set_coordinate_lut(d, tab.table, **kw)
    ps = _pixel_screen(inst)
    pid, toa = synthetic.dream_events(1_000_000, inst, seed=3)
    eng.stage(pid, toa)
    eng.accumulate(0)
    eng.set_coordinate_lut(d + 0.1, tab.table, **kw)
    eng.stage(pid, toa)
    eng.accumulate(1)
    res = eng.finalize(hists=True)
    pix = ora.pixel_index(pid, inst.detector_number)
    exp = np.zeros_like(res.current_hist)
    for r, shift in ((0, 0.0), (1, 0.1)):
        c = ora.wavelength_mode(lt + shift, tab.table, tab.distance0, tab.distance_step,
                                tab.time0, tab.time_step)(pix, toa)
        exp += ora.detector_histogram(ps[r], view.n_screen, pix, c, edges)
    np.testing.assert_array_equal(res.current_hist, exp)


def test_workflow_wavelength_mode_and_move():
    """``coordinate_mode='wavelength'`` through GpuDetectorViewFactory: the
    spectral coord is 'wavelength' in the edges' unit, the images match the
    oracle, and a detector move re-projects and recomputes Ltotal."""
    from esslivedata_amd import geometry, synthetic, wavelength
    from esslivedata_amd.edges import WavelengthEdges
    from esslivedata_amd.workflows import (DetectorViewParams, GeometricViewConfig,
                                           GpuDetectorViewFactory)

    inst = synthetic.loki_bank0(n_replicas=1)
    off = inst.positions - [0.0, 0.0, 5.0]
    res = inst.resolution
    src = (0.0, 0.0, -23.0)
    tab = wavelength.ideal_lookup_table(27.5, 29.5, 41, 71.5e6, 287)
    fac = GpuDetectorViewFactory(
        detector_numbers={'loki': inst.detector_number},
        view_config=GeometricViewConfig('xy_plane', res),
        positions={'loki': off}, transforms={'loki': np.array([0.0, 0.0, 5.0])},
        lookup_table=tab, source_position=src)
    wl = WavelengthEdges(start=1.0, stop=10.0, num_bins=60)
    params = DetectorViewParams(coordinate_mode='wavelength', wavelength_edges=wl,
                                wavelength_range=(2.0, 6.0))
    wf = fac.make_workflow('loki', params)
    pid, toa = synthetic.uniform_events(1_000_000, 1, 802816, seed=4)
    t0 = np.eye(4)
    t0[2, 3] = 5.0
    t1 = t0.copy()
    t1[2, 3] = 6.0  # moved 1 m downstream: longer flight paths
    lo, hi = ora.label_slice(wl.get_edges(), 2.0, 6.0)
    for step, tr in enumerate([t0, t1]):
        wf.accumulate({'loki': (pid, toa), 'detector_transform': tr}, start_time=_t(step),
                      end_time=_t(step + 1))
        h = wf.read_histogram('current')
        out = wf.finalize()
        pos = geometry.apply_transform(tr, off)
        ps = ora.geometric_pixel_screen(geometry.make_xy_plane_coords(pos), res)
        lt = wavelength.pixel_ltotal(pos, source_position=src)
        pix = ora.pixel_index(pid, inst.detector_number)
        c = ora.wavelength_mode(lt, tab.table, tab.distance0, tab.distance_step, tab.time0,
                                tab.time_step)(pix, toa)
        exp = ora.detector_histogram(ps[0], 144 * 144, pix, c, wl.get_edges())
        assert h.dims == ('y', 'x', 'wavelength')
        assert h.coords['wavelength'].unit == 'Å'
        np.testing.assert_array_equal(h.coords['wavelength'].values, wl.get_edges())
        np.testing.assert_array_equal(h.values.reshape(144 * 144, -1), exp)
        np.testing.assert_array_equal(out['current'].values,
                                      exp[:, lo:hi].sum(-1).reshape(144, 144))
        assert float(out['counts_in_toa_range'].values) == exp[:, lo:hi].sum()


@pytest.mark.parametrize('unit', ['Å', 'nm'])
def test_monitor_wavelength_mode(unit):
    """``histogram_wavelength_monitor`` (monitor_workflow.py:126-132): every
    event at the monitor's flight path through the table, binned on the
    wavelength edges; the coord is the edges in the event unit and back."""
    from esslivedata_amd import synthetic
    from esslivedata_amd.edges import WavelengthEdges, convert_wavelength
    from esslivedata_amd.workflows import create_gpu_monitor_workflow

    tab = synthetic.dream_wavelength_table()
    wl = (WavelengthEdges(start=0.5, stop=3.5, num_bins=100) if unit == 'Å'
          else WavelengthEdges(start=0.05, stop=0.35, num_bins=100, unit='nm'))
    wf = create_gpu_monitor_workflow('monitor_1', wl, range_filter=None,
                                     coordinate_mode='wavelength', lookup_table=tab,
                                     monitor_distance=77.85)
    rng = np.random.default_rng(8)
    toa = rng.normal(30e6, 12e6, 2_000_000).astype(np.int32)
    wf.accumulate({'monitor_1': (None, toa)}, start_time=_t(0), end_time=_t(1))
    out = wf.finalize()
    e_ev = wl.edges_in('Å')
    c = ora.coordinate_lookup(np.full(toa.size, 77.85), toa, tab.table, tab.distance0,
                              tab.distance_step, tab.time0, tab.time_step)
    exp = ora.monitor_histogram(c, e_ev)
    np.testing.assert_array_equal(out['current'].values, exp)
    assert out['current'].dims == ('wavelength',)
    np.testing.assert_array_equal(out['current'].coords['wavelength'].values,
                                  convert_wavelength(e_ev, 'Å', unit))
    assert float(out['counts_total'].values) == exp.sum()


@pytest.mark.parametrize('strategy', ['atomic', 'split', 'wide'])
@pytest.mark.parametrize('kind', ['duplicates', 'many_bins'])
def test_coordinate_bins_for_unusual_edges(kind, strategy):
    """Edges with empty (repeated) bins, and 20000 bins (edges too large for
    LDS: read from HBM): the bucketed search still gives scipp's bins."""
    from esslivedata_amd import projection
    from esslivedata_amd.engine import BinningEngine

    if kind == 'duplicates':
        edges = np.sort(np.concatenate([np.linspace(1.0, 9.0, 41), [2.0, 2.0, 5.5, 7.25]]))
    else:
        edges = np.geomspace(0.5, 9.5, 20001)
    rng = np.random.default_rng(12)
    nd, nt, dt = 6, 40, 2048.0
    tab = rng.uniform(0.4, 9.6, (nd, nt))
    tab[:, ::7] = edges[rng.integers(0, edges.size, (nd, (nt + 6) // 7))]  # exact edge values
    dn = np.arange(1, 65, dtype=np.int32)
    view = projection.logical_lut(dn)
    ltot = (np.arange(64) % nd) * 0.5 + 3.0
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy)
    eng.set_coordinate_lut(ltot, tab, dist0=3.0, dist_step=0.5, time0=0.0, time_step=dt)
    n = 300_000
    pid = rng.integers(1, 65, n).astype(np.int32)
    toa = rng.integers(-10, int(dt) * nt + 10, n).astype(np.int32)
    toa[: n // 2] = (toa[: n // 2] // int(dt)) * int(dt)  # on time nodes: exact table values
    eng.stage(pid, toa)
    eng.accumulate(0)
    res = eng.finalize(hists=True)
    o = ora.OracleDetectorView(dn, np.arange(64)[None], (64,), edges,
                               coordinate=ora.wavelength_mode(ltot, tab, 3.0, 0.5, 0.0, dt))
    o.accumulate(pid, toa)
    np.testing.assert_array_equal(res.current_hist, o.finalize()['histogram_current'])


@pytest.mark.parametrize('strategy', ['pixel', 'auto'])
def test_loki_wavelength_on_pixel_matches_oracle(strategy):
    """PIXEL after the coordinate pre-pass: LOKI bank 0, whose
    footprints fit LDS, in wavelength mode.  The pre-pass writes every
    event's coordinate bin as its "time"; PIXEL then bins those against the
    integer edges 0..T with the tables sized at create time.  Three batches
    (counted, then predicted slots) over two replicas, bit-exact against the
    NumPy oracle, and PIXEL is what ran."""
    from esslivedata_amd import projection, synthetic, wavelength
    from esslivedata_amd.edges import WavelengthEdges
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.loki_bank0(n_replicas=2)
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    tab = wavelength.ideal_lookup_table(27.5, 29.5, 41, 71.5e6, 287)
    lt = wavelength.pixel_ltotal(inst.positions, source_position=(0.0, 0.0, -23.0))
    d = wavelength.distance_per_pid(inst.detector_number, lt, view.pid_offset, view.lut.shape[1])
    edges = WavelengthEdges(start=0.5, stop=10.0, num_bins=100).get_edges()
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy)
    eng.set_coordinate_lut(d, tab.table, dist0=tab.distance0, dist_step=tab.distance_step,
                           time0=tab.time0, time_step=tab.time_step)
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number, pixel_screen=_pixel_screen(inst),
        screen_shape=tuple(view.screen_shape), toa_edges_ns=edges,
        coordinate=ora.wavelength_mode(lt, tab.table, tab.distance0, tab.distance_step,
                                       tab.time0, tab.time_step))
    for batch in range(3):
        pid, toa = synthetic.uniform_events(1_500_001 + batch, 1, 802816, seed=500 + batch)
        eng.stage(pid[:600_000], toa[:600_000])
        eng.stage(pid[600_000:], toa[600_000:])
        eng.accumulate(batch % 2)
        assert eng.info()['last_strategy'] == 'pixel'
        o.accumulate(pid, toa)
    res = eng.finalize(hists=True)
    exp = o.finalize()
    assert exp['histogram_cumulative'].sum() > 3_000_000
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
