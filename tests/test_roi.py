"""ROI spectra and spectrum views on the CPU: the oracle against the reference's
own ROI test expectations, and the host-side group construction
(``esslivedata_amd.roi`` / ``projection.index_groups``) against the oracle.

Reference tests restated: tests/workflows/detector_view/roi_test.py:127-380
(10x10 screen over 0..10 m, uniform histogram of ones with 3 TOF bins)."""

import numpy as np
import pytest

from oracle import scipp_semantics as ora

EDGES = np.linspace(0.0, 10.0, 11)
CENTERS = 0.5 * (EDGES[1:] + EDGES[:-1])


def _view(with_coords=True):
    from esslivedata_amd.projection import ViewLUT

    kw = {}
    if with_coords:
        kw = dict(screen_coords={'y': CENTERS, 'x': CENTERS}, screen_edges={'y': EDGES, 'x': EDGES},
                  screen_units={'y': 'm', 'x': 'm'})
    return ViewLUT(pid_offset=0, lut=np.zeros((1, 1), np.int32), screen_shape=(10, 10),
                   screen_dims=('y', 'x'), **kw)


def _ones(nt=3):
    return np.ones((10, 10, nt))


def _host_spectra(view, hist, rects, polys):
    """Group sums of the host-built screen groups (what the GPU sums)."""
    from esslivedata_amd import roi

    idx, groups = roi.roi_groups(view, rects, polys)
    flat = hist.reshape(-1, hist.shape[-1])
    return idx, np.asarray([flat[g].sum(axis=0) for g in groups]).reshape(len(groups), hist.shape[-1])


def _case(rects=None, polys=None, with_coords=True, hist=None):
    from esslivedata_amd import roi

    rects = rects or {}
    polys = polys or {}
    view = _view(with_coords)
    hist = _ones() if hist is None else hist
    o_rects = [((r.y.min, r.y.max, r.y.unit), (r.x.min, r.x.max, r.x.unit)) for r in rects.values()]
    xc = CENTERS if with_coords else np.arange(10.0)
    o_polys = [
        ora.polygon_inside(p.x, p.y, xc if p.x_unit else np.arange(10.0),
                           xc if p.y_unit else np.arange(10.0))
        for p in polys.values()
    ]
    exp = ora.roi_spectra(hist, o_rects, o_polys, EDGES, EDGES)
    idx, got = _host_spectra(view, hist, rects, polys)
    assert idx == list(rects) + list(polys)
    np.testing.assert_array_equal(got.reshape(exp.shape), exp)
    _ = roi
    return exp


def test_rectangle_physical_coords():  # roi_test.py:127-146
    from esslivedata_amd.roi import Interval, RectangleROI

    r = RectangleROI(x=Interval(2.0, 5.0, 'm'), y=Interval(2.0, 5.0, 'm'))
    np.testing.assert_array_equal(_case({0: r})[0], [9, 9, 9])


def test_rectangle_index_bounds():  # roi_test.py:148-164
    from esslivedata_amd.roi import Interval, RectangleROI

    r = RectangleROI(x=Interval(0, 5), y=Interval(0, 5))
    np.testing.assert_array_equal(_case({0: r})[0], [25, 25, 25])


def test_rectangle_none_coords():  # roi_test.py:166-182
    from esslivedata_amd.roi import Interval, RectangleROI

    r = RectangleROI(x=Interval(2, 5), y=Interval(2, 5))
    np.testing.assert_array_equal(_case({0: r}, with_coords=False)[0], [9, 9, 9])


def test_multiple_rectangles():  # roi_test.py:184-208
    from esslivedata_amd.roi import Interval, RectangleROI

    rects = {0: RectangleROI(x=Interval(0, 2, 'm'), y=Interval(0, 2, 'm')),
             1: RectangleROI(x=Interval(5, 10, 'm'), y=Interval(5, 10, 'm'))}
    exp = _case(rects)
    np.testing.assert_array_equal(exp, [[4, 4, 4], [25, 25, 25]])


def test_polygon_square_edges_and_centers():  # roi_test.py:211-257
    from esslivedata_amd.roi import PolygonROI

    p = PolygonROI(x=[2.0, 5.0, 5.0, 2.0], y=[2.0, 2.0, 5.0, 5.0], x_unit='m', y_unit='m')
    np.testing.assert_array_equal(_case(polys={0: p})[0], [9, 9, 9])


def test_polygon_none_coords():  # roi_test.py:259-283
    from esslivedata_amd.roi import PolygonROI

    p = PolygonROI(x=[1.5, 4.5, 4.5, 1.5], y=[1.5, 1.5, 4.5, 4.5])
    np.testing.assert_array_equal(_case(polys={0: p}, with_coords=False)[0], [9, 9, 9])


def test_triangle_polygon():  # roi_test.py:285-322
    from esslivedata_amd.roi import PolygonROI

    hist = np.zeros((10, 10, 3))
    for y in range(10):
        hist[y] = y
    p = PolygonROI(x=[0.0, 10.0, 0.0], y=[0.0, 0.0, 10.0], x_unit='m', y_unit='m')
    exp = _case(polys={0: p}, hist=hist)
    assert 0 < exp.sum() < 1350 * 0.75


def test_rectangles_and_polygons_together():  # roi_test.py:325-356
    from esslivedata_amd.roi import Interval, PolygonROI, RectangleROI

    rects = {0: RectangleROI(x=Interval(0, 2, 'm'), y=Interval(0, 2, 'm'))}
    polys = {100: PolygonROI(x=[5.0, 10.0, 10.0, 5.0], y=[5.0, 5.0, 10.0, 10.0],
                             x_unit='m', y_unit='m')}
    exp = _case(rects, polys)
    assert exp.shape == (2, 3)
    np.testing.assert_array_equal(exp[0], [4, 4, 4])


def test_empty_requests():  # roi_test.py:361-380
    from esslivedata_amd import roi

    assert _case().shape == (0, 3)
    assert roi.from_concatenated(roi.to_concatenated({}, 'rectangle')) == {}
    assert roi.from_concatenated(roi.to_concatenated({}, 'polygon')) == {}
    assert roi.from_concatenated(None) == {}


def test_wire_form_round_trip_and_errors():
    from esslivedata_amd.roi import (Interval, PolygonROI, RectangleROI, from_concatenated,
                                     rectangle_screens, to_concatenated)

    rects = {3: RectangleROI(x=Interval(1, 2, 'm'), y=Interval(0.5, 7, 'm')),
             0: RectangleROI(x=Interval(0, 4, 'm'), y=Interval(2, 3, 'm'))}
    da = to_concatenated(rects, 'rectangle')
    assert da.dims == ('bounds',) and list(da.coords['roi_index'].values) == [0, 0, 3, 3]
    assert from_concatenated(da) == rects
    polys = {1: PolygonROI(x=[0, 1, 1], y=[0, 0, 1], x_unit='mm', y_unit='mm')}
    assert from_concatenated(to_concatenated(polys, 'polygon')) == polys
    with pytest.raises(ValueError):  # one request, one unit (sc.concat)
        to_concatenated({0: RectangleROI(x=Interval(0, 1, 'm'), y=Interval(0, 1, 'm')),
                         1: RectangleROI(x=Interval(0, 1), y=Interval(0, 1))})
    empty = to_concatenated({}, 'rectangle', coord_units={'x': 'm', 'y': 'm'})
    assert empty.coords['x'].unit == 'm' and empty.values.size == 0
    with pytest.raises(ValueError):
        Interval(2, 1)
    with pytest.raises(ValueError):
        PolygonROI(x=[0, 1], y=[0, 1])
    # label-based rectangle with a unit that does not match the screen coord
    with pytest.raises(ValueError):
        rectangle_screens(_view(), RectangleROI(x=Interval(0, 1, 's'), y=Interval(0, 1, 's')))
    # polygon in mm against a screen in m: centers are converted (roi.py:165-171)
    from esslivedata_amd.roi import polygon_screens

    p_mm = PolygonROI(x=[2000.0, 5000.0, 5000.0, 2000.0], y=[2000.0, 2000.0, 5000.0, 5000.0],
                      x_unit='mm', y_unit='mm')
    assert len(polygon_screens(_view(), p_mm)) == 9


def test_label_slice_on_random_geometry_matches_oracle():
    """Rectangles with arbitrary physical bounds on non-integer edges."""
    from esslivedata_amd.projection import ViewLUT
    from esslivedata_amd.roi import Interval, RectangleROI, roi_groups

    rng = np.random.default_rng(5)
    ye, xe = np.linspace(-1.3, 2.7, 81), np.linspace(0.1, 5.2, 321)
    view = ViewLUT(pid_offset=0, lut=np.zeros((1, 1), np.int32), screen_shape=(80, 320),
                   screen_dims=('arc_length', 'z'), screen_edges={'arc_length': ye, 'z': xe},
                   screen_coords={'arc_length': 0.5 * (ye[1:] + ye[:-1]), 'z': 0.5 * (xe[1:] + xe[:-1])},
                   screen_units={'arc_length': 'm', 'z': 'm'})
    hist = rng.integers(0, 50, (80, 320, 7)).astype(np.float64)
    rects = {}
    for i in range(12):
        y0, y1 = np.sort(rng.uniform(-2, 3, 2))
        x0, x1 = np.sort(rng.uniform(-0.5, 6, 2))
        rects[i] = RectangleROI(x=Interval(x0, x1, 'm'), y=Interval(y0, y1, 'm'))
    exp = ora.roi_spectra(hist, [((r.y.min, r.y.max, 'm'), (r.x.min, r.x.max, 'm'))
                                 for r in rects.values()], [], ye, xe)
    idx, groups = roi_groups(view, rects, {})
    flat = hist.reshape(-1, 7)
    got = np.asarray([flat[g].sum(axis=0) for g in groups])
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize('ppt', [1, 4, 10, 100])
def test_bifrost_spectrum_groups_match_oracle(ppt):
    from esslivedata_amd import projection, synthetic

    cfg = synthetic.bifrost_spectrum_config(ppt)
    shape, groups = projection.index_groups((15, 900), cfg.transform, cfg.reduction_axes)
    assert shape == (5, 27 * ppt)
    rng = np.random.default_rng(ppt)
    hist = rng.integers(0, 1000, (15, 900, 11)).astype(np.float32)
    exp = ora.bifrost_spectrum_view(hist.astype(np.float64), ppt)
    flat = hist.reshape(-1, 11).astype(np.float64)
    got = np.asarray([flat[g].sum(axis=0) for g in groups]).reshape(*shape, 11)
    np.testing.assert_array_equal(got, exp)
