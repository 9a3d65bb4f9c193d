"""CPU oracle: a NumPy restatement of the reference's event-binning hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / CPU baseline.  The product path (``esslivedata_amd``) never imports
it: binning always runs on the HIP engine and fails loudly without it.

What is restated (reference = /root/reference, SRC = src/ess/livedata):

* TOA edges: ``make_edges`` -> ``sc.linspace``/``sc.geomspace`` (numpy under the
  hood), SRC/parameter_models.py:290-295; converted to the event unit with
  ``bins.to(unit=event_unit)`` (ms -> ns, one f64 multiply by 1e6),
  SRC/workflows/detector_view/providers.py:205-207 and
  SRC/workflows/monitor_workflow.py:93-95.
* scipp ``hist``: half-open bins ``[e_i, e_{i+1})`` including the last one,
  int32 event coordinate compared against float64 edges, out-of-range and NaN
  dropped (providers.py:208, monitor_workflow.py:97).
* ``group_event_data``: events whose ``event_id`` is not a value of the
  flattened ``detector_number`` are dropped; pixel index = row-major position
  (SRC/preprocessors/group_by_pixel.py:36-54, _patch_group_event_data.py:23-35).
* ``GeometricProjector``: one replica per ``project_events`` call, cycling
  ``counter % R`` (SRC/workflows/detector_view/projectors.py:105-113); per-event
  screen coordinate gather (:123-143) then ``bin(edges)`` (:152); screen edges
  ``coords[dim].hist({dim: res}).coords[dim]`` (:344-350) = scipp's
  int-bin-count rule ``linspace(nanmin, nextafter(nanmax, +inf), res + 1)``;
  ``flip_x`` negates x (:341-342).
* ``LogicalProjector``: transform (reshape/slice) then ``bins.concat`` over the
  reduction dims (projectors.py:243-270); restated as an index-array transform.
* Accumulators: cumulative ``NoCopyAccumulator`` (first push copies, then
  ``+=``, reset when the scalar reset coord changes) and the window
  accumulator cleared on finalize (SRC/preprocessors/accumulators.py:86-195).
* Finalize outputs: ``detector_image`` (sum over the spectral dim, optional
  label slice), ``counts_total``, ``counts_in_range``
  (providers.py:236-357); monitor ``counts_total``/``counts_in_range``
  (monitor_workflow.py:147-167); output target names
  (detector_view/factory.py:208-215, monitor_workflow.py:318-325).

Scipp rules that cannot be verified offline (scipp is not installed) are pinned
by the hand-derived known-answer tests in ``tests/test_oracle_kat.py`` and by
the reference's own test expectations; see DESIGN.md "Parity".
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Sequence

import numpy as np

# ESS_PULSE_PERIOD_MS, SRC/parameter_models.py:26
ESS_PULSE_PERIOD_MS = float(np.ceil(1000.0 / 14 * 100) / 100)

# scipp unit conversion factors for time units -> ns (f64 multiply).
_TO_NS = {'ns': 1.0, 'us': 1e3, 'μs': 1e3, 'ms': 1e6, 's': 1e9}


# --------------------------------------------------------------------------
# Edges
# --------------------------------------------------------------------------
def make_edges(start: float, stop: float, num_bins: int, scale: str = 'linear'):
    """``make_edges`` (SRC/parameter_models.py:290-295): linspace/geomspace."""
    if scale == 'linear':
        return np.linspace(start, stop, num_bins + 1)
    if scale == 'log':
        return np.geomspace(start, stop, num_bins + 1)
    raise ValueError(f"unknown scale {scale!r}")


def to_ns(edges: np.ndarray, unit: str) -> np.ndarray:
    """``edges.to(unit='ns')`` as one f64 multiply (providers.py:207)."""
    factor = _TO_NS[unit]
    edges = np.asarray(edges, dtype=np.float64)
    return edges if factor == 1.0 else edges * factor


def hist_bin_index(values: np.ndarray, edges: np.ndarray) -> np.ndarray:
    """Bin index of each value under scipp's ``hist`` rule; -1 = dropped.

    Half-open ``[e_i, e_{i+1})`` for every bin including the last, comparison
    in float64 (int32 TOA promoted exactly), NaN dropped.
    """
    v = np.asarray(values)
    vf = v.astype(np.float64, copy=False)
    idx = np.searchsorted(edges, vf, side='right') - 1
    nb = len(edges) - 1
    bad = (idx < 0) | (idx >= nb)
    if vf.dtype.kind == 'f':
        bad |= np.isnan(vf)
    idx = idx.astype(np.int64)
    idx[bad] = -1
    return idx


def label_slice(edges: np.ndarray, low: float, high: float) -> tuple[int, int]:
    """Bin range selected by scipp label slicing ``da[dim, low:high]`` on a
    bin-edge coordinate: from the bin containing ``low`` to the bins that
    overlap ``[low, high)``.  Pinned by the KAT at
    tests/workflows/monitor_workflow_test.py:233-243 (edges 0..10 ns / 6,
    [2 ns, 8 ns) -> bins 1..3)."""
    nb = len(edges) - 1
    begin = int(np.searchsorted(edges, low, side='right')) - 1
    end = int(np.searchsorted(edges, high, side='left'))
    return max(begin, 0), min(max(end, 0), nb)


def screen_edges(coord_all_replicas: np.ndarray, res: int) -> np.ndarray:
    """scipp ``Variable.hist({dim: res})`` edge rule (projectors.py:344-350):
    ``linspace(nanmin, nextafter(nanmax, +inf), res + 1)`` over all replicas."""
    lo = float(np.nanmin(coord_all_replicas))
    hi = float(np.nanmax(coord_all_replicas))
    return np.linspace(lo, np.nextafter(hi, np.inf), res + 1)


# --------------------------------------------------------------------------
# Pixel grouping and projection (LUT construction is setup-time)
# --------------------------------------------------------------------------
def pixel_index(event_id: np.ndarray, detector_number: np.ndarray) -> np.ndarray:
    """``group_event_data`` membership: row-major pixel index or -1 (dropped)."""
    dn = np.asarray(detector_number).ravel()
    order = np.argsort(dn, kind='stable')
    sdn = dn[order]
    pos = np.searchsorted(sdn, event_id)
    pos_c = np.minimum(pos, len(sdn) - 1)
    hit = (pos < len(sdn)) & (sdn[pos_c] == event_id)
    out = np.full(len(event_id), -1, dtype=np.int64)
    out[hit] = order[pos_c[hit]]
    return out


def geometric_screen_index(
    coords: dict[str, np.ndarray], edges: dict[str, np.ndarray], replica: int
) -> np.ndarray:
    """Flat screen index per pixel for one replica (-1 = outside / NaN).

    ``coords[dim]`` has shape ``(R, P)``; dims in ``edges`` order (the order of
    the ``resolution`` dict, projectors.py:345-350) are row-major.
    """
    dims = list(edges)
    flat = None
    for dim in dims:
        b = hist_bin_index(np.asarray(coords[dim])[replica], edges[dim])
        n = len(edges[dim]) - 1
        if flat is None:
            flat = b.copy()
        else:
            bad = (flat < 0) | (b < 0)
            flat = flat * n + b
            flat[bad] = -1
    return flat


def geometric_pixel_screen(
    coords: dict[str, np.ndarray], resolution: dict[str, int], flip_x: bool = False
) -> np.ndarray:
    """``(R, P)`` screen index per replica and pixel of a geometric view:
    ``flip_x`` negates x (projectors.py:341-342), edges over all replicas
    (:344-350), dims in ``resolution`` order."""
    c = dict(coords)
    if flip_x and 'x' in c:
        c['x'] = -np.asarray(c['x'])
    edges = {d: screen_edges(c[d], r) for d, r in resolution.items()}
    n_rep = np.asarray(next(iter(c.values()))).shape[0]
    return np.stack([geometric_screen_index(c, edges, k) for k in range(n_rep)])


def logical_screen_index(
    detector_shape: Sequence[int],
    transform: Callable[[np.ndarray], np.ndarray] | None,
    reduction_axes: Sequence[int] = (),
) -> tuple[np.ndarray, tuple[int, ...]]:
    """Output index per pixel for a logical view (projectors.py:243-270).

    The transform is applied to an index-valued array shaped like the
    detector; pixels that the transform drops (slicing) get -1; reduced axes
    are merged (``bins.concat``).  Returns ``(lut[P], output_shape)``.
    """
    p = int(np.prod(detector_shape))
    idx = np.arange(p, dtype=np.int64).reshape(detector_shape)
    t = idx if transform is None else transform(idx)
    t = np.asarray(t)
    kept = [a for a in range(t.ndim) if a not in set(reduction_axes)]
    out_shape = tuple(t.shape[a] for a in kept)
    moved = np.moveaxis(t, kept, list(range(len(kept))))
    n_out = int(np.prod(out_shape)) if out_shape else 1
    moved = moved.reshape(n_out, -1)
    lut = np.full(p, -1, dtype=np.int64)
    for o in range(n_out):
        lut[moved[o]] = o
    return lut, out_shape


def folded_view_index(
    sizes: dict[str, int],
    out_axes: Sequence[Sequence[str]],
    fixed: dict[str, int] | None = None,
) -> tuple[np.ndarray, tuple[int, ...]]:
    """Closed-form output index per pixel of a fold / transpose / slice /
    flatten / ``bins.concat`` logical view (projectors.py:243-270), derived
    without applying any transform: pixel ``p`` has mixed-radix coordinates
    over ``sizes`` (row-major ``fold``, dict order slowest first); it is kept
    when every ``fixed`` dim equals its value (``['wire', 0]``); its output
    index is the mixed-radix number over ``out_axes`` (each a group of dims
    flattened in the given order, e.g. ``('module', 'segment', 'counter')``);
    dims in neither are merged.  Used for the DREAM views
    (config/instruments/dream/views.py:13-85) and MAGIC views
    (config/instruments/magic/views.py:38-85)."""
    fixed = dict(fixed or {})
    names = list(sizes)
    radix = [int(sizes[d]) for d in names]
    p = int(np.prod(radix))
    coord = {}
    rem = np.arange(p, dtype=np.int64)
    for d, n in zip(reversed(names), reversed(radix)):
        coord[d] = rem % n
        rem = rem // n
    keep = np.ones(p, dtype=bool)
    for d, v in fixed.items():
        keep &= coord[d] == int(v)
    out = np.zeros(p, dtype=np.int64)
    shape = []
    for group in out_axes:
        n_group = 1
        g = np.zeros(p, dtype=np.int64)
        for d in group:
            g = g * sizes[d] + coord[d]
            n_group *= sizes[d]
        out = out * n_group + g
        shape.append(n_group)
    out[~keep] = -1
    return out, tuple(shape)


# --------------------------------------------------------------------------
# Histograms
# --------------------------------------------------------------------------
def detector_histogram(
    pixel_screen: np.ndarray,
    n_screen: int,
    event_pixel: np.ndarray,
    toa: np.ndarray,
    toa_edges_ns: np.ndarray,
    dtype=np.float64,
) -> np.ndarray:
    """One batch: group -> project -> ``hist`` over TOA (providers.py:169-214).

    ``event_pixel`` is the pixel index per event (-1 = unknown id) and
    ``pixel_screen`` the screen index per pixel (-1 = off screen).
    Returns ``(n_screen, T)`` counts in ``dtype`` (f64, or f32 for BIFROST).
    """
    t = len(toa_edges_ns) - 1
    ok = event_pixel >= 0
    scr = np.full(len(event_pixel), -1, dtype=np.int64)
    scr[ok] = pixel_screen[event_pixel[ok]]
    tb = hist_bin_index(toa, toa_edges_ns)
    keep = (scr >= 0) & (tb >= 0)
    flat = scr[keep] * t + tb[keep]
    counts = np.bincount(flat, minlength=n_screen * t)
    return counts.reshape(n_screen, t).astype(dtype)


def coordinate_lookup(distance: np.ndarray, toa: np.ndarray, table: np.ndarray,
                      dist0: float, dist_step: float, time0: float,
                      time_step: float) -> np.ndarray:
    """Wavelength-mode event coordinate (detector_view/factory.py:134-169,
    providers.py:77-95): bilinear lookup of ``table`` (n_dist x n_time) at the
    event's pixel distance and time of arrival; NaN where the distance is NaN
    or either point lies outside the grid.

    essreduce's ``GenericUnwrapWorkflow`` (the table's producer and
    interpolator) is not in /root/reference, so this restates the documented
    engine arithmetic (include/lde.h ``lde_set_coord_lut``) step for step in
    float64 -- numpy evaluates each ``a + f * (b - a)`` as a rounded product
    then a rounded sum, the unfused order the kernel is compiled to.  Parity
    with the reference's own table interpolation is unpinned.
    """
    tab = np.asarray(table, dtype=np.float64)
    nd, nt = tab.shape
    d = np.asarray(distance, dtype=np.float64)
    x = (d - dist0) * (1.0 / dist_step)
    okx = (x >= 0.0) & (x <= nd - 1)
    i = np.minimum(np.floor(np.where(okx, x, 0.0)), nd - 2).astype(np.int64)
    fx = x - i
    y = (np.asarray(toa).astype(np.float64) - time0) * (1.0 / time_step)
    oky = (y >= 0.0) & (y <= nt - 1)
    j = np.minimum(np.floor(np.where(oky, y, 0.0)), nt - 2).astype(np.int64)
    fy = y - j
    v00 = tab[i, j]
    v01 = tab[i, j + 1]
    v10 = tab[i + 1, j]
    v11 = tab[i + 1, j + 1]
    a = v00 + fy * (v01 - v00)
    b = v10 + fy * (v11 - v10)
    c = a + fx * (b - a)
    return np.where(okx & oky, c, np.nan)


def wavelength_mode(ltotal: np.ndarray, table: np.ndarray, dist0: float, dist_step: float,
                    time0: float, time_step: float) -> Callable:
    """``OracleDetectorView.coordinate`` for wavelength mode: each event's
    pixel ``Ltotal`` (row-major pixel order) and TOA -> ``coordinate_lookup``."""
    lt = np.asarray(ltotal, dtype=np.float64).ravel()

    def coordinate(pix: np.ndarray, toa: np.ndarray) -> np.ndarray:
        d = np.where(pix >= 0, lt[np.maximum(pix, 0)], np.nan)
        return coordinate_lookup(d, toa, table, dist0, dist_step, time0, time_step)

    return coordinate


def monitor_histogram(toa: np.ndarray, toa_edges_ns: np.ndarray) -> np.ndarray:
    """``_histogram_monitor`` event mode (monitor_workflow.py:90-100)."""
    tb = hist_bin_index(toa, toa_edges_ns)
    tb = tb[tb >= 0]
    return np.bincount(tb, minlength=len(toa_edges_ns) - 1).astype(np.float64)


def rebin(src_edges: np.ndarray, values: np.ndarray, dst_edges: np.ndarray) -> np.ndarray:
    """``_histogram_monitor`` histogram mode (monitor_workflow.py:101-108):
    scipp ``rebin`` of a 1-D float64 histogram, uniform density inside each
    source bin; each new bin sums ``value * overlap / width`` over the source
    bins in ascending order.  Pinned by the reference's KATs
    (tests/workflows/monitor_workflow_test.py:190-216, 518-548); the exact
    rounding order beyond them is parity unpinned (scipp's C++ rebin)."""
    se = np.asarray(src_edges, dtype=np.float64)
    sv = np.asarray(values, dtype=np.float64)
    de = np.asarray(dst_edges, dtype=np.float64)
    out = np.zeros(len(de) - 1)
    for j in range(len(de) - 1):
        lo, hi = de[j], de[j + 1]
        acc = 0.0
        for i in range(len(sv)):
            xl, xh = se[i], se[i + 1]
            ov = min(xh, hi) - max(xl, lo)
            if ov > 0.0:
                acc += sv[i] * ov / (xh - xl)
        out[j] = acc
    return out


# --------------------------------------------------------------------------
# Accumulator pair (accumulators.py:86-195)
# --------------------------------------------------------------------------
@dataclass
class AccumulatorPair:
    """Cumulative (copy on first push, ``+=``) + window (cleared on finalize),
    both resetting when the pushed value's geometry coord differs."""

    cumulative: np.ndarray | None = None
    window: np.ndarray | None = None
    cum_geom: object = None
    win_geom: object = None

    @staticmethod
    def _changed(stored, new) -> bool:
        return stored is not None and new is not None and stored != new

    def push(self, value: np.ndarray, geometry=None) -> None:
        if self.cumulative is not None and self._changed(self.cum_geom, geometry):
            self.cumulative = None
        if self.cumulative is None:
            self.cumulative = value.copy()
        else:
            self.cumulative += value
        self.cum_geom = geometry
        if self.window is not None and self._changed(self.win_geom, geometry):
            self.window = None
        if self.window is None:
            self.window = value.copy()
        else:
            self.window += value
        self.win_geom = geometry

    def on_finalize(self) -> None:
        self.window = None
        self.win_geom = None

    def clear(self) -> None:
        self.cumulative = None
        self.window = None
        self.cum_geom = None
        self.win_geom = None


# --------------------------------------------------------------------------
# ROI spectra and spectrum views (finalize-side regroupings)
# --------------------------------------------------------------------------
def roi_rectangle_slice(n: int, bounds, edges: np.ndarray | None) -> slice:
    """One axis of ``histogram[dim, low:high]`` (roi.py:221-228): integer bounds
    (``Interval.to_bounds`` without unit, SRC/config/models.py:274-290) slice
    positionally, physical bounds slice by label on the bin-edge coord."""
    low, high, unit = bounds
    if unit is None:
        return slice(int(low), int(high))
    b, e = label_slice(edges, low, high)
    return slice(b, e)


def polygon_inside(xs, ys, x_centers: np.ndarray, y_centers: np.ndarray) -> np.ndarray:
    """``_compute_polygon_mask`` (roi.py:128-185) without the inversion:
    matplotlib ``Path.contains_points`` on the (y, x) grid of bin centers."""
    from matplotlib.path import Path

    xx, yy = np.meshgrid(x_centers, y_centers)
    path = Path(list(zip(xs, ys)))
    return path.contains_points(np.column_stack([xx.ravel(), yy.ravel()])).reshape(xx.shape)


def roi_spectra(hist: np.ndarray, rectangles: Sequence, polygons: Sequence,
                y_edges: np.ndarray | None = None, x_edges: np.ndarray | None = None) -> np.ndarray:
    """``roi_spectra`` (roi.py:188-266) on a dense ``(y, x, spectral)`` array:
    rectangles (``(y_bounds, x_bounds)`` with bounds ``(low, high, unit)``)
    first, then polygons (``(y, x)`` boolean inside masks), each summed over
    both screen dims -> ``(n_roi, spectral)``."""
    ny, nx, nt = hist.shape
    out = []
    for yb, xb in rectangles:
        sy = roi_rectangle_slice(ny, yb, y_edges)
        sx = roi_rectangle_slice(nx, xb, x_edges)
        out.append(hist[sy][:, sx].sum(axis=(0, 1)))
    for inside in polygons:
        out.append(hist[inside].sum(axis=0))  # masked sum: outside bins excluded
    return np.asarray(out, dtype=hist.dtype).reshape(len(out), nt)


def bifrost_spectrum_view(hist: np.ndarray, pixels_per_tube: int = 10) -> np.ndarray:
    """``_bifrost_spectrum_transform`` (bifrost/specs.py:311-329) on a dense
    ``(arc/tube=15, channel/pixel=900, toa)`` array: fold arc/tube -> (arc 5,
    tube 3), channel/pixel -> (channel 9, pixel 100), pixel -> (pixel,
    subpixel), sum subpixel, flatten (tube, channel, pixel) -> detector_number."""
    sub = 100 // pixels_per_tube
    nt = hist.shape[-1]
    h = hist.reshape(5, 3, 9, pixels_per_tube, sub, nt).sum(axis=4)
    return h.reshape(5, 3 * 9 * pixels_per_tube, nt)


# --------------------------------------------------------------------------
# Workflow-level restatements
# --------------------------------------------------------------------------
@dataclass
class OracleDetectorView:
    """Detector-view workflow semantics (factory.py:95-276, providers.py)."""

    detector_number: np.ndarray
    pixel_screen: np.ndarray  # (R, P) screen index per replica and pixel
    screen_shape: tuple[int, ...]
    toa_edges_ns: np.ndarray
    toa_slice: tuple[int, int] | None = None  # bin range of HistogramSlice
    dtype: type = np.float64
    # wavelength mode: (pixel index, toa) -> event coordinate, binned on
    # ``toa_edges_ns`` (then in the coordinate's unit); see wavelength_mode()
    coordinate: Callable | None = None
    _counter: int = 0
    _acc: AccumulatorPair = field(default_factory=AccumulatorPair)

    @property
    def n_screen(self) -> int:
        return int(np.prod(self.screen_shape))

    def batch_histogram(self, pid, toa, replica: int) -> np.ndarray:
        pix = pixel_index(np.asarray(pid), self.detector_number)
        values = np.asarray(toa)
        if self.coordinate is not None:
            values = self.coordinate(pix, values)
        return detector_histogram(
            self.pixel_screen[replica],
            self.n_screen,
            pix,
            values,
            self.toa_edges_ns,
            self.dtype,
        )

    def accumulate(self, pid, toa, geometry=None) -> None:
        r = self._counter % self.pixel_screen.shape[0]
        self._counter += 1
        self._acc.push(self.batch_histogram(pid, toa, r), geometry)

    def _outputs(self, hist: np.ndarray) -> dict:
        lo, hi = self.toa_slice if self.toa_slice else (0, hist.shape[-1])
        img = hist[:, lo:hi].sum(axis=-1).reshape(self.screen_shape)
        return {
            'image': img,
            'total': hist.sum(),
            'in_range': hist[:, lo:hi].sum(),
        }

    def finalize(self) -> dict:
        if self._acc.cumulative is None:
            raise ValueError("No data has been added")
        cum = self._outputs(self._acc.cumulative)
        cur = self._outputs(self._acc.window)
        out = {
            'cumulative': cum['image'],
            'current': cur['image'],
            'counts_total': cur['total'],
            'counts_in_toa_range': cur['in_range'],
            'counts_total_cumulative': cum['total'],
            'counts_in_toa_range_cumulative': cum['in_range'],
            'histogram_cumulative': self._acc.cumulative.copy(),
            'histogram_current': self._acc.window.copy(),
        }
        self._acc.on_finalize()
        return out

    def clear(self) -> None:
        self._acc.clear()


@dataclass
class OracleMonitor:
    """Monitor-histogram workflow semantics (monitor_workflow.py:65-331)."""

    toa_edges_ns: np.ndarray
    range_slice: tuple[int, int] | None = None
    _acc: AccumulatorPair = field(default_factory=AccumulatorPair)

    def accumulate(self, toa, geometry=None) -> None:
        self._acc.push(monitor_histogram(np.asarray(toa), self.toa_edges_ns), geometry)

    def finalize(self) -> dict:
        if self._acc.cumulative is None:
            raise ValueError("No data has been added")
        lo, hi = self.range_slice if self.range_slice else (0, len(self.toa_edges_ns) - 1)
        cum, cur = self._acc.cumulative, self._acc.window
        out = {
            'cumulative': cum.copy(),
            'current': cur.copy(),
            'counts_total': cur.sum(),
            'counts_in_toa_range': cur[lo:hi].sum(),
            'counts_total_cumulative': cum.sum(),
            'counts_in_toa_range_cumulative': cum[lo:hi].sum(),
        }
        self._acc.on_finalize()
        return out

    def clear(self) -> None:
        self._acc.clear()
