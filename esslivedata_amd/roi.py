"""ROI requests -> screen groups for the device-side ROI spectra.

Setup-time host code, run when an ROI request arrives (the reference
precomputes bounds and masks at the same moment,
SRC/workflows/detector_view/roi.py:31-125).  The per-finalize reduction
``(screen..., toa) -> (roi, toa)`` runs on the GPU (``lde_group_spectra``);
this module only decides which flat screen indices belong to each ROI.

Mirrored reference behaviour:

* models: ``Interval`` / ``RectangleROI`` / ``PolygonROI`` and the
  concatenated wire form with a ``roi_index`` coord, ROI type encoded in the
  dim name ``bounds`` / ``vertex`` (SRC/config/models.py:82-240, 255-460);
* rectangles (roi.py:31-70, 221-228): ``y_dim, x_dim = dims[0], dims[1]`` of
  the screen; bounds with a unit slice the histogram by label on its screen
  coord (bin edges for geometric views -> the bins overlapping
  ``[min, max)``; a unit mismatch raises as scipp does); bounds without a unit
  are positional ``[int(min):int(max)]``;
* polygons (roi.py:73-173): point-in-polygon of the screen-bin centers
  (converted to the ROI unit) with ``matplotlib.path.Path.contains_points``;
  without a unit, or for logical views without coords, centers are
  ``arange(n)``.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Mapping, Union

import numpy as np

from .dataarray import DataArray, Variable
from .edges import label_slice
from .projection import ViewLUT

_LENGTH_TO_M = {'m': 1.0, 'cm': 1e-2, 'mm': 1e-3, 'um': 1e-6, 'µm': 1e-6, 'nm': 1e-9}


@dataclass(frozen=True)
class Interval:
    """``models.Interval`` (SRC/config/models.py:255-290)."""

    min: float
    max: float
    unit: str | None = None

    def __post_init__(self) -> None:
        if self.min >= self.max:
            raise ValueError(f'min ({self.min}) must be < max ({self.max})')


@dataclass(frozen=True)
class RectangleROI:
    """``models.RectangleROI`` (SRC/config/models.py:293-360)."""

    x: Interval
    y: Interval


@dataclass(frozen=True)
class PolygonROI:
    """``models.PolygonROI`` (SRC/config/models.py:363-420)."""

    x: tuple[float, ...]
    y: tuple[float, ...]
    x_unit: str | None = None
    y_unit: str | None = None

    def __post_init__(self) -> None:
        object.__setattr__(self, 'x', tuple(float(v) for v in self.x))
        object.__setattr__(self, 'y', tuple(float(v) for v in self.y))
        if len(self.x) != len(self.y):
            raise ValueError('x and y must have the same length')
        if len(self.x) < 3:
            raise ValueError('Polygon must have at least 3 vertices')


ROI = Union[RectangleROI, PolygonROI]


# ---------------------------------------------------------------------------
# wire form (models.ROI.to/from_concatenated_data_array, models.py:148-223)
# ---------------------------------------------------------------------------
def to_concatenated(rois: Mapping[int, ROI], kind: str = 'rectangle',
                    coord_units: Mapping[str, str | None] | None = None) -> DataArray:
    """Concatenate ROIs along ``bounds`` (rectangles) or ``vertex`` (polygons)."""
    dim = {'rectangle': 'bounds', 'polygon': 'vertex'}[kind]
    xs, ys, idx = [], [], []
    xu = yu = None
    for i in sorted(rois):
        r = rois[i]
        if isinstance(r, RectangleROI):
            if dim != 'bounds':
                raise TypeError('rectangle ROI in a polygon request')
            xs += [r.x.min, r.x.max]
            ys += [r.y.min, r.y.max]
            xu, yu = r.x.unit, r.y.unit
            idx += [i, i]
        else:
            if dim != 'vertex':
                raise TypeError('polygon ROI in a rectangle request')
            xs += list(r.x)
            ys += list(r.y)
            xu, yu = r.x_unit, r.y_unit
            idx += [i] * len(r.x)
    units = {(r.x.unit, r.y.unit) if isinstance(r, RectangleROI) else (r.x_unit, r.y_unit)
             for r in rois.values()}
    if len(units) > 1:  # sc.concat of coords with different units raises
        raise ValueError(f'ROIs of one request must share coordinate units, got {sorted(map(str, units))}')
    if not rois and coord_units:
        xu, yu = coord_units.get('x'), coord_units.get('y')
    return DataArray(
        np.ones(len(xs), dtype=np.int32), (dim,), '',
        {
            'x': Variable((dim,), np.asarray(xs, dtype=np.float64), xu),
            'y': Variable((dim,), np.asarray(ys, dtype=np.float64), yu),
            'roi_index': Variable((dim,), np.asarray(idx, dtype=np.int32)),
        },
    )


def from_concatenated(da: DataArray | Mapping[int, ROI] | None) -> dict[int, ROI]:
    """Parse a concatenated request (or pass a ``{index: ROI}`` dict through)."""
    if da is None:
        return {}
    if isinstance(da, Mapping):
        return dict(da)
    if len(np.atleast_1d(da.values)) == 0:
        return {}
    dim = da.dims[0]
    idx = np.asarray(da.coords['roi_index'].values)
    x, y = np.asarray(da.coords['x'].values), np.asarray(da.coords['y'].values)
    xu, yu = da.coords['x'].unit, da.coords['y'].unit
    out: dict[int, ROI] = {}
    for i in np.unique(idx):
        sel = idx == i
        if dim == 'bounds':
            xv, yv = x[sel], y[sel]
            out[int(i)] = RectangleROI(Interval(float(xv[0]), float(xv[1]), xu),
                                       Interval(float(yv[0]), float(yv[1]), yu))
        elif dim == 'vertex':
            out[int(i)] = PolygonROI(tuple(x[sel]), tuple(y[sel]), xu, yu)
        else:
            raise ValueError(f'Cannot determine ROI type from dimension: {dim}')
    return out


# ---------------------------------------------------------------------------
# ROI -> flat screen indices
# ---------------------------------------------------------------------------
def _screen_axes(view: ViewLUT) -> tuple[str, str]:
    if len(view.screen_dims) != 2:
        raise ValueError(f'Expected 2 spatial dims, got {len(view.screen_dims)}: {view.screen_dims}')
    return view.screen_dims[0], view.screen_dims[1]


def _convert(values: np.ndarray, unit: str | None, to: str | None) -> np.ndarray:
    if unit == to:
        return values
    if unit in _LENGTH_TO_M and to in _LENGTH_TO_M:
        return values * (_LENGTH_TO_M[unit] / _LENGTH_TO_M[to])
    raise ValueError(f'cannot convert coordinate unit {unit!r} to {to!r}')


def _axis_range(view: ViewLUT, dim: str, axis: int, iv: Interval) -> tuple[int, int]:
    n = view.screen_shape[axis]
    if iv.unit is None:  # positional (Interval.to_bounds, models.py:274-290)
        lo, hi = int(iv.min), int(iv.max)
        lo = min(max(lo, 0), n)
        return lo, min(max(hi, lo), n)
    edges = view.screen_edges.get(dim)
    if edges is None:
        raise ValueError(f'screen dim {dim!r} has no coordinate for a label-based ROI')
    unit = view.screen_units.get(dim)
    if unit != iv.unit:
        raise ValueError(f'ROI unit {iv.unit!r} does not match the {dim!r} coord unit {unit!r}')
    return label_slice(np.asarray(edges, dtype=np.float64), float(iv.min), float(iv.max))


def rectangle_screens(view: ViewLUT, roi: RectangleROI) -> np.ndarray:
    """Flat screen indices of ``histogram[y, y0:y1][x, x0:x1]`` (roi.py:221-228)."""
    y_dim, x_dim = _screen_axes(view)
    y0, y1 = _axis_range(view, y_dim, 0, roi.y)
    x0, x1 = _axis_range(view, x_dim, 1, roi.x)
    grid = np.arange(view.n_screen, dtype=np.int64).reshape(view.screen_shape)
    return grid[y0:y1, x0:x1].ravel().astype(np.int32)


def _centers(view: ViewLUT, dim: str, axis: int, unit: str | None) -> np.ndarray:
    n = view.screen_shape[axis]
    coord = view.screen_coords.get(dim)
    if unit is None:  # roi.py:157-165: pixel indices
        return np.arange(n, dtype=np.float64)
    if coord is None:  # roi.py:104-110: logical view, synthesized (dimensionless) indices
        raise ValueError(f'screen dim {dim!r} has no coordinate to convert to {unit!r}')
    return _convert(np.asarray(coord, dtype=np.float64), view.screen_units.get(dim), unit)


def polygon_mask_inside(view: ViewLUT, roi: PolygonROI) -> np.ndarray:
    """Boolean ``(y, x)`` array: screen-bin centers inside the polygon
    (``_compute_polygon_mask``, roi.py:128-185, without the inversion)."""
    from matplotlib.path import Path

    y_dim, x_dim = _screen_axes(view)
    xv = _centers(view, x_dim, 1, roi.x_unit)
    yv = _centers(view, y_dim, 0, roi.y_unit)
    xx, yy = np.meshgrid(xv, yv)
    path = Path(list(zip(roi.x, roi.y)))
    inside = path.contains_points(np.column_stack([xx.ravel(), yy.ravel()]))
    return inside.reshape(xx.shape)


def polygon_screens(view: ViewLUT, roi: PolygonROI) -> np.ndarray:
    inside = polygon_mask_inside(view, roi)
    return np.flatnonzero(inside.ravel()).astype(np.int32)


def roi_groups(view: ViewLUT, rectangles: Mapping[int, ROI],
               polygons: Mapping[int, ROI]) -> tuple[list[int], list[np.ndarray]]:
    """ROI indices (rectangles first, then polygons, as ``roi_spectra`` stacks
    them, roi.py:218-236) and their flat screen-index groups."""
    idx: list[int] = []
    groups: list[np.ndarray] = []
    for i, r in rectangles.items():
        if isinstance(r, RectangleROI):
            idx.append(int(i))
            groups.append(rectangle_screens(view, r))
    for i, r in polygons.items():
        if isinstance(r, PolygonROI):
            idx.append(int(i))
            groups.append(polygon_screens(view, r))
    return idx, groups
