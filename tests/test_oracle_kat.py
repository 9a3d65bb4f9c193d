"""Pin the CPU oracle against the reference's known answers (CPU only).

The reference itself cannot be imported in this container (it needs Python
>= 3.12 and scipp/essreduce, which are absent -- ordinary errors, not a
permission denial), so the oracle is pinned by the KATs transcribed from the
reference's own tests (tests/golden/reference_kats.json) and by hand-derived
edge-tie cases (tests/golden/tie_kats.json).
"""

import json
from pathlib import Path

import numpy as np
import pytest

from oracle import scipp_semantics as ora

GOLDEN = Path(__file__).resolve().parent / 'golden'
REF = {k['name']: k for k in json.loads((GOLDEN / 'reference_kats.json').read_text())}
TIES = json.loads((GOLDEN / 'tie_kats.json').read_text())


@pytest.mark.parametrize(
    'name', ['group_by_pixel_sizes', 'group_by_pixel_two_messages', 'group_by_pixel_after_get']
)
def test_group_by_pixel_kats(name):
    kat = REF[name]
    dn = np.array(kat['detector_number'])
    pid = np.concatenate([m['pixel_id'] for m in kat['messages']])
    pix = ora.pixel_index(pid, dn)
    sizes = np.bincount(pix[pix >= 0], minlength=len(dn))
    np.testing.assert_array_equal(sizes, kat['expected_sizes'])


def test_group_by_pixel_drops_unknown_and_noncontiguous_ids():
    dn = np.array([[7, 3], [11, 100]])  # folded, non-contiguous (dream high-res style)
    pid = np.array([3, 3, 4, 100, 7, 0, 11, 101])
    np.testing.assert_array_equal(ora.pixel_index(pid, dn), [1, 1, -1, 3, 0, -1, 2, -1])


def test_monitor_histogram_kat():
    kat = REF['monitor_event_histogram']
    h = ora.monitor_histogram(np.array(kat['toa_ns'], np.int32), np.array(kat['edges_ns']))
    assert h.sum() == kat['expected_sum']
    np.testing.assert_array_equal(h, kat['expected_hist'])


def test_monitor_cumulative_window_kat():
    """monitor_workflow_test.py:484-516 through the oracle's accumulator pair:
    the cumulative keeps both cycles, the window only the last."""
    kat = REF['monitor_cumulative_accumulates_window_clears']
    h = ora.monitor_histogram(np.array(kat['toa_ns'], np.int32), np.array(kat['edges_ns']))
    cum = np.zeros_like(h)
    for exp in kat['expected']:
        cum = cum + h
        assert cum.sum() == exp['cumulative_sum']
        assert h.sum() == exp['current_sum']


def test_counts_in_range_kat():
    kat = REF['monitor_counts_in_range']
    lo, hi = ora.label_slice(np.array(kat['edges_ns']), *kat['range_ns'])
    assert (lo, hi) == (1, 4)
    assert np.sum(np.array(kat['hist'])[lo:hi]) == kat['expected']
    assert np.sum(REF['monitor_counts_total']['hist']) == REF['monitor_counts_total']['expected']


def test_label_slice_rule():
    edges = np.array([0.0, 2.0, 4.0, 6.0, 8.0, 10.0])
    assert ora.label_slice(edges, 1.0, 7.0) == (0, 4)  # bins containing / overlapping
    assert ora.label_slice(edges, 0.0, 10.0) == (0, 5)
    assert ora.label_slice(edges, -5.0, 50.0) == (0, 5)
    assert ora.label_slice(edges, 4.0, 4.0) == (2, 2)


def test_accumulator_pair_service_kat():
    """detector_data_test.py:57-131: 2000 -> 2000/2000, +3000 -> 5000/3000,
    +1000+1000 -> 7000/2000 on the dummy panel."""
    kat = REF['detector_service_cumulative_current']
    dn = np.arange(1, 128**2 + 1).reshape(128, 128)
    edges = np.linspace(0, ora.ESS_PULSE_PERIOD_MS, 101) * 1e6
    o = ora.OracleDetectorView(
        detector_number=dn,
        pixel_screen=np.arange(128**2)[None, :],
        screen_shape=(128, 128),
        toa_edges_ns=edges,
    )
    rng = np.random.default_rng(1234)
    for sizes, cum, cur in zip(kat['batches'], kat['expected_cumulative'], kat['expected_current']):
        for n in sizes:  # each message is its own accumulate call in the service
            toa = rng.uniform(0, 70_000_000, n).astype(np.int32)
            pid = rng.integers(1, 128**2 + 1, n, dtype=np.int32)
            o.accumulate(pid, toa)
        out = o.finalize()
        assert np.nansum(out['cumulative']) == cum
        assert np.nansum(out['current']) == cur
        assert out['counts_total'] == cur and out['counts_total_cumulative'] == cum


def test_accumulator_reset_on_geometry_change():
    """accumulators.py:116-131: a changed reset coord restarts the cumulative."""
    acc = ora.AccumulatorPair()
    acc.push(np.array([1.0, 2.0]), geometry='g1')
    acc.on_finalize()
    acc.push(np.array([1.0, 1.0]), geometry='g1')
    np.testing.assert_array_equal(acc.cumulative, [2.0, 3.0])
    acc.on_finalize()
    acc.push(np.array([5.0, 0.0]), geometry='g2')
    np.testing.assert_array_equal(acc.cumulative, [5.0, 0.0])
    np.testing.assert_array_equal(acc.window, [5.0, 0.0])
    acc.push(np.array([1.0, 1.0]), geometry=None)  # absent coord: no reset
    np.testing.assert_array_equal(acc.cumulative, [6.0, 1.0])


@pytest.mark.parametrize('kat', TIES['toa'], ids=lambda k: k['name'])
def test_toa_edge_ties(kat):
    if 'edges_ms' in kat:
        spec = kat['edges_ms']
        op = {'linspace': np.linspace, 'geomspace': np.geomspace}[spec['op']]
        edges = ora.to_ns(op(spec['start'], spec['stop'], spec['num']), 'ms')
        for i, v in kat['f64_edges_ns_used'].items():
            assert edges[int(i)] == v  # pins linspace/geomspace + ms->ns f64 arithmetic
    else:
        edges = np.array(kat['edges_ns'])
    toa = np.array([c[0] for c in kat['cases']], dtype=np.int32)
    exp = np.array([c[1] for c in kat['cases']])
    np.testing.assert_array_equal(ora.hist_bin_index(toa, edges), exp)


@pytest.mark.parametrize('kat', TIES['screen'], ids=lambda k: k['name'])
def test_screen_edge_rule(kat):
    v = np.array(kat['values'], dtype=np.float64)
    e = ora.screen_edges(v, kat['res'])
    np.testing.assert_array_equal(ora.hist_bin_index(v, e), kat['expected_bins'])


def test_oracle_regression_vector():
    """Restatement-generated golden vector (tests/golden/dream_small.npz)."""
    from esslivedata_amd import synthetic

    g = np.load(GOLDEN / 'dream_small.npz')
    inst = synthetic.dream_mantle()
    edges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    ps = ora.geometric_screen_index(inst.coords, edges, int(g['replica']))
    pix = ora.pixel_index(g['pid'], inst.detector_number)
    hist = ora.detector_histogram(ps, 25600, pix, g['toa'], inst.edges.edges_ns()).ravel()
    nz = np.nonzero(hist)[0]
    np.testing.assert_array_equal(nz, g['hist_index'])
    np.testing.assert_array_equal(hist[nz], g['hist_value'])


def test_logical_view_reduction_and_slicing():
    # fold 4x6 -> transpose, drop column 0, merge axis 0
    lut, shape = ora.logical_screen_index((4, 6), lambda a: a.T[1:], reduction_axes=(1,))
    assert shape == (5,)
    idx = np.arange(24).reshape(4, 6)
    for r in range(4):
        assert lut[idx[r, 0]] == -1
        for c in range(1, 6):
            assert lut[idx[r, c]] == c - 1


def test_c_oracle_matches_numpy_oracle():
    """oracle/binning_ref.c (the CPU baseline) restates the same rules."""
    from esslivedata_amd import synthetic
    from oracle import c_oracle

    g = np.load(GOLDEN / 'dream_small.npz')
    inst = synthetic.dream_mantle()
    edges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    ps = np.stack([ora.geometric_screen_index(inst.coords, edges, k) for k in range(2)])
    c = c_oracle.CDetectorView(inst.detector_number, ps, 25600, inst.edges.edges_ns(), threads=4)
    h = c.accumulate(g['pid'], g['toa'], int(g['replica']))
    nz = np.nonzero(h)[0]
    np.testing.assert_array_equal(nz, g['hist_index'])
    np.testing.assert_array_equal(h[nz], g['hist_value'])
    # edge-tie KATs through the C binary search
    for kat in TIES['toa']:
        if 'edges_ns' not in kat:
            continue
        e = np.array(kat['edges_ns'])
        cv = c_oracle.CDetectorView(np.array([1]), np.array([[0]]), 1, e, threads=1)
        toa = np.array([x[0] for x in kat['cases']], dtype=np.int32)
        exp = np.array([x[1] for x in kat['cases']])
        got = cv.accumulate(np.ones(len(toa), np.int32), toa)
        np.testing.assert_array_equal(got, np.bincount(exp[exp >= 0], minlength=len(e) - 1))


def test_rebin_kats_from_the_reference_monitor_tests():
    """monitor_workflow_test.py:190-216 (sums preserved; 0..10 ns in 10 bins
    onto linspace(0, 10, 6)) and :518-548 (ten ones -> total 10)."""
    dst = np.linspace(0, 10, 6)
    vals = [1.0, 2.0, 3.0, 4.0, 5.0, 4.0, 3.0, 2.0, 1.0, 0.0]
    got = ora.rebin(np.linspace(0, 10, 11), vals, dst)
    np.testing.assert_array_equal(got, [3.0, 7.0, 9.0, 5.0, 1.0])
    assert got.sum() == sum(vals)
    assert ora.rebin(np.linspace(0, 10, 11), [1.0] * 10, dst).sum() == 10.0
    # partial overlaps: uniform density, outside the target range dropped
    got = ora.rebin(np.array([-1.0, 1.0, 3.0]), [2.0, 4.0], np.array([0.0, 2.0, 4.0]))
    np.testing.assert_array_equal(got, [1.0 + 2.0, 2.0])


# ---------------------------------------------------------------------------
# round 2: projector, accumulator and monitor-workflow KATs (reference tests
# transcribed as data, tests/golden/make_golden.py:reference_kats_r2)
# ---------------------------------------------------------------------------
DEFAULT_TOA_NS = np.linspace(0, 71.43, 101) * 1e6


def _projector_counts(kat, replica):
    coords = {d: np.array(v) for d, v in kat['coords'].items()}
    edges = {d: np.array(v) for d, v in kat['edges'].items()}
    ps = ora.geometric_screen_index(coords, edges, replica)
    pix = ora.pixel_index(np.array(kat['events']['event_id']), np.array(kat['detector_number']))
    n = int(np.prod([len(e) - 1 for e in edges.values()]))
    return ora.detector_histogram(ps, n, pix, np.array(kat['events']['toa']), DEFAULT_TOA_NS)


def test_projector_count_conservation_kat():
    kat = REF['projector_count_conservation']
    assert _projector_counts(kat, kat['replica']).sum() == kat['expected_total']


def test_projector_replicas_differ_kat():
    kat = REF['projector_replicas_differ']
    a = _projector_counts(kat, 0).sum(-1)
    b = _projector_counts(kat, 1).sum(-1)
    assert not np.array_equal(a, b)


def test_projector_flip_x_kat_through_geometry_builder():
    from esslivedata_amd import geometry

    kat = REF['projector_flip_x_mirrors']
    coords = geometry.make_xy_plane_coords(np.array(kat['positions']))
    res = kat['resolution']
    pix = ora.pixel_index(np.array(kat['events']['event_id']), np.array(kat['detector_number']))
    imgs = {}
    for flip in (False, True):
        ps = ora.geometric_pixel_screen(coords, res, flip_x=flip)
        h = ora.detector_histogram(ps[0], 6, pix, np.array(kat['events']['toa']), DEFAULT_TOA_NS)
        imgs[flip] = h.sum(-1).reshape(res['x'], res['y'])
    n_x = res['x']
    for i in range(n_x):
        np.testing.assert_array_equal(imgs[True][i], imgs[False][n_x - 1 - i])
    assert imgs[False].sum() == 300
    np.testing.assert_array_equal(ora.screen_edges(coords['y'], 2),
                                  ora.screen_edges(geometry.make_xy_plane_coords(
                                      np.array(kat['positions']))['y'], 2))


def test_accumulator_pair_kats():
    kat = REF['accumulator_window_accumulates']
    acc = ora.AccumulatorPair()
    for p in kat['pushes']:
        acc.push(np.array(p, dtype=float))
    np.testing.assert_array_equal(acc.window, kat['expected_window'])

    acc = ora.AccumulatorPair()
    acc.push(np.array(REF['accumulator_window_cleared_on_finalize']['pushes'][0], dtype=float))
    acc.on_finalize()
    assert acc.window is None

    kat = REF['accumulator_pair_multiple_cycles']
    acc = ora.AccumulatorPair()
    for h in kat['cycles']:
        acc.push(np.array(h, dtype=float))
        np.testing.assert_array_equal(acc.window, h)
        acc.on_finalize()
    np.testing.assert_array_equal(acc.cumulative, kat['expected_cumulative'])

    kat = REF['accumulator_pair_multiple_pushes_per_window']
    acc = ora.AccumulatorPair()
    for n, w in zip(kat['n_pushes'], kat['expected_windows']):
        for j in range(n):
            acc.push(np.array([j, j + 1], dtype=float))
        np.testing.assert_array_equal(acc.window, w)
        acc.on_finalize()
    np.testing.assert_array_equal(acc.cumulative, kat['expected_cumulative'])

    for case in REF['accumulator_reset_on_coord_change']['cases']:
        acc = ora.AccumulatorPair()
        for vals, coord in case['pushes']:
            acc.push(np.array(vals, dtype=float), coord)
        if 'expected_cumulative' in case:
            np.testing.assert_array_equal(acc.cumulative, case['expected_cumulative'])
        else:
            np.testing.assert_array_equal(acc.window, case['expected_window'])


def test_monitor_full_workflow_cycle_kat():
    kat = REF['monitor_full_workflow_cycle']
    o = ora.OracleMonitor(np.array(kat['edges_ns']))
    o.accumulate(np.array(kat['toa_ns'], dtype=np.int32))
    out = o.finalize()
    exp = kat['expected']
    assert out['cumulative'].sum() == exp['cumulative_sum']
    assert out['current'].sum() == exp['current_sum']
    for k in ('counts_total', 'counts_in_toa_range', 'counts_total_cumulative',
              'counts_in_toa_range_cumulative'):
        assert out[k] == exp[k]
