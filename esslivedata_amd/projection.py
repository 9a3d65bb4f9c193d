"""Setup-time construction of the engine's pid -> screen lookup tables.

This is host code that runs once per job / geometry (like the reference's
projector construction at job creation); the per-event work runs
on the GPU.  It folds three reference steps into one int32 table per noise
replica:

* ``group_event_data`` membership and pixel index
  (SRC/preprocessors/group_by_pixel.py:36-54): ids not in ``detector_number``
  map to -1 (dropped); pixel index = row-major position.
* geometric projection (SRC/workflows/detector_view/projectors.py:306-352):
  per-replica screen coordinates binned with scipp's int-bin-count edge rule
  ``linspace(nanmin, nextafter(nanmax, +inf), res + 1)``; half-open bins; NaN
  and out-of-range -> -1; ``flip_x`` negates ``x``; screen dims follow the
  order of the ``resolution`` dict.
* logical projection (projectors.py:243-270): a reshape/slice transform of
  the detector array followed by merging of reduction dims; computed by
  applying the transform to an index array.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Sequence

import numpy as np

from .logical import LogicalIndex, detector_index, reduction_dims

MAX_LUT_LEN = 1 << 28


@dataclass
class ViewLUT:
    """Per-replica pid -> flat screen index table for :class:`BinningEngine`."""

    pid_offset: int
    lut: np.ndarray  # (R, L) int32, -1 = dropped
    screen_shape: tuple[int, ...]
    screen_dims: tuple[str, ...]
    screen_coords: dict[str, np.ndarray] = field(default_factory=dict)
    screen_edges: dict[str, np.ndarray] = field(default_factory=dict)
    pixel_weights: np.ndarray | None = None
    screen_units: dict[str, str | None] = field(default_factory=dict)

    @property
    def n_screen(self) -> int:
        return int(np.prod(self.screen_shape)) if self.screen_shape else 1

    @property
    def n_replicas(self) -> int:
        return self.lut.shape[0]


def pid_pixel_table(detector_number: np.ndarray) -> tuple[int, np.ndarray]:
    """Dense ``pid - pid_offset -> pixel index`` table (-1 = unknown id)."""
    dn = np.asarray(detector_number).ravel().astype(np.int64)
    if dn.size == 0:
        raise ValueError('detector_number is empty')
    lo, hi = int(dn.min()), int(dn.max())
    length = hi - lo + 1
    if length > MAX_LUT_LEN:
        raise ValueError(f'detector_number range {length} too large for a dense LUT')
    if lo < -(2**31) or hi >= 2**31:
        raise ValueError('detector numbers must fit in int32')
    table = np.full(length, -1, dtype=np.int64)
    pos = dn - lo
    if len(np.unique(pos)) != len(pos):
        raise ValueError('detector_number contains duplicate ids')
    table[pos] = np.arange(dn.size, dtype=np.int64)
    return lo, table


def scipp_hist_edges(values: np.ndarray, res: int) -> np.ndarray:
    """scipp's edges for ``hist({dim: res})`` with an integer bin count."""
    lo = float(np.nanmin(values))
    hi = float(np.nanmax(values))
    return np.linspace(lo, np.nextafter(hi, np.inf), int(res) + 1)


def _bin_half_open(values: np.ndarray, edges: np.ndarray) -> np.ndarray:
    idx = np.searchsorted(edges, values, side='right') - 1
    bad = (idx < 0) | (idx >= len(edges) - 1) | np.isnan(values)
    idx = idx.astype(np.int64)
    idx[bad] = -1
    return idx


def _compose(detector_number, pixel_screen: np.ndarray) -> tuple[int, np.ndarray]:
    """LUT[r][pid - off] = pixel_screen[r][pixel(pid)]."""
    off, table = pid_pixel_table(detector_number)
    known = table >= 0
    lut = np.full((pixel_screen.shape[0], len(table)), -1, dtype=np.int32)
    lut[:, known] = pixel_screen[:, table[known]]
    return off, lut


def geometric_lut(
    detector_number: np.ndarray,
    coords: dict[str, np.ndarray],
    resolution: dict[str, int] | None = None,
    *,
    flip_x: bool = False,
    unit: str = 'm',
    edges: dict[str, np.ndarray] | None = None,
) -> ViewLUT:
    """LUT for a geometric view from per-replica projected coordinates.

    ``coords[dim]`` has shape ``(R, P)`` (replica, detector pixel), as produced
    by essreduce's ``make_xy_plane_coords`` / ``make_cylinder_mantle_coords``
    on ``CalibratedPositionWithNoisyReplicas``.  Screen edges follow scipp's
    rule for ``resolution`` (make_geometric_projector, projectors.py:344-350),
    or are given explicitly (``GeometricProjector(coords, edges)``,
    projectors.py:45-78), dims in dict order.
    """
    coords = {k: np.atleast_2d(np.asarray(v, dtype=np.float64)) for k, v in coords.items()}
    if flip_x and 'x' in coords:
        coords['x'] = -coords['x']
    if edges is not None:
        edges = {d: np.asarray(e, dtype=np.float64) for d, e in edges.items()}
        resolution = {d: len(e) - 1 for d, e in edges.items()}
    if resolution is None:
        raise ValueError('geometric_lut needs a resolution or explicit edges')
    dims = tuple(resolution)
    p = int(np.asarray(detector_number).size)
    for d in dims:
        if d not in coords:
            raise ValueError(f'no projected coordinate for screen dim {d!r}')
        if coords[d].shape[1] != p:
            raise ValueError(f'coordinate {d!r} has {coords[d].shape[1]} pixels, expected {p}')
    if edges is None:
        edges = {d: scipp_hist_edges(coords[d], resolution[d]) for d in dims}
    shape = tuple(int(resolution[d]) for d in dims)
    r = coords[dims[0]].shape[0]
    pixel_screen = np.empty((r, p), dtype=np.int64)
    for rep in range(r):
        flat = None
        for d, n in zip(dims, shape):
            b = _bin_half_open(coords[d][rep], edges[d])
            if flat is None:
                flat = b
            else:
                bad = (flat < 0) | (b < 0)
                flat = flat * n + b
                flat[bad] = -1
        pixel_screen[rep] = flat
    off, lut = _compose(detector_number, pixel_screen)
    # pixel weights: mean number of pixels per screen bin over replicas
    # (GeometricProjector.compute_weights, projectors.py:154-172), float32
    w = np.zeros(int(np.prod(shape)), dtype=np.float64)
    for rep in range(r):
        ok = pixel_screen[rep] >= 0
        w += np.bincount(pixel_screen[rep][ok], minlength=len(w))
    weights = (w.astype(np.float32) / np.float32(r)).reshape(shape)
    return ViewLUT(
        pid_offset=off,
        lut=lut,
        screen_shape=shape,
        screen_dims=dims,
        screen_coords={d: 0.5 * (edges[d][1:] + edges[d][:-1]) for d in dims},
        screen_edges=edges,
        pixel_weights=weights,
        screen_units={d: unit for d in dims},
    )


def _reduce_axes(t, reduction_axes: Sequence[int],
                 reduction_dim: str | Sequence[str] | None) -> tuple[np.ndarray, list[int], tuple]:
    """Transformed index array, the kept axes and their names (None when
    the transform returned a plain array)."""
    names = t.dims if isinstance(t, LogicalIndex) else None
    arr = np.asarray(t.values if isinstance(t, LogicalIndex) else t)
    red = set(int(a) % arr.ndim for a in reduction_axes) if arr.ndim else set()
    rdims = reduction_dims(reduction_dim)
    if rdims:
        if names is None:
            raise ValueError('reduction_dim needs a transform that keeps dim names '
                             '(fold/flatten on the LogicalIndex it receives)')
        for d in rdims:
            if d not in names:
                raise ValueError(f'reduction dim {d!r} not in the transformed dims {names}')
            red.add(names.index(d))
    kept = [a for a in range(arr.ndim) if a not in red]
    kept_names = None if names is None else tuple(names[a] for a in kept)
    return arr, kept, kept_names


def logical_lut(
    detector_number: np.ndarray,
    *,
    dims: Sequence[str] | None = None,
    transform: Callable[[np.ndarray], np.ndarray] | None = None,
    output_dims: Sequence[str] | None = None,
    reduction_axes: Sequence[int] = (),
    reduction_dim: str | Sequence[str] | None = None,
) -> ViewLUT:
    """LUT for a logical view (identity, fold/flatten/slice, reduction).

    ``transform`` receives a :class:`LogicalIndex` (pixel indices shaped like
    ``detector_number``, dims ``dims`` or ``('detector_number',)`` for 1-D) and
    returns the folded / transposed / sliced / flattened result, as the
    reference's transforms do to the detector data
    (LogicalProjector.project_events, projectors.py:243-270); pixels it drops
    map to -1.  The named ``reduction_dim`` (projectors.py:186-207), or the
    positional ``reduction_axes`` of a transform returning a plain array, are
    merged (``bins.concat``).  Output dims are the kept names.
    """
    dn = np.asarray(detector_number)
    p = dn.size
    idx = detector_index(dn, dims)
    t = idx if transform is None else transform(idx)
    arr, kept, kept_names = _reduce_axes(t, reduction_axes, reduction_dim)
    out_shape = tuple(arr.shape[a] for a in kept)
    moved = np.moveaxis(arr, kept, list(range(len(kept)))) if arr.ndim else arr
    n_out = int(np.prod(out_shape)) if out_shape else 1
    moved = moved.reshape(n_out, -1)
    if moved.size and (moved.min() < 0 or moved.max() >= p):
        raise ValueError('the transform produced indices outside the detector')
    if moved.size != len(np.unique(moved)):
        raise ValueError('the transform duplicated detector pixels')
    pix_out = np.full(p, -1, dtype=np.int64)
    out_ids = np.repeat(np.arange(n_out, dtype=np.int64), moved.shape[1])
    pix_out[moved.ravel()] = out_ids
    off, lut = _compose(dn, pix_out[None, :])
    weights = np.bincount(pix_out[pix_out >= 0], minlength=n_out).astype(np.float32)
    if output_dims is None:
        if kept_names is not None:
            output_dims = kept_names
        else:
            output_dims = tuple(f'dim_{i}' for i in range(len(out_shape)))
    if len(tuple(output_dims)) != len(out_shape):
        raise ValueError(f'output_dims {tuple(output_dims)} do not match the view shape {out_shape}')
    return ViewLUT(
        pid_offset=off,
        lut=lut,
        screen_shape=out_shape,
        screen_dims=tuple(output_dims),
        pixel_weights=weights.reshape(out_shape),
    )


def index_groups(
    shape: Sequence[int],
    transform: Callable[[np.ndarray], np.ndarray] | None = None,
    reduction_axes: Sequence[int] = (),
) -> tuple[tuple[int, ...], list[np.ndarray]]:
    """Output groups of a sum-preserving regrouping of a ``shape`` grid.

    ``transform`` gets the flat-index array of shape ``shape`` and returns it
    folded / transposed / sliced; ``reduction_axes`` of the result are summed.
    Returns the output shape and, per output element (row-major), the flat
    input indices it sums.  Used for spectrum views, whose transforms
    fold + sum + flatten the screen dims (SRC/workflows/detector_view/
    providers.py:300-325, bifrost/specs.py:311-329).
    """
    idx = np.arange(int(np.prod(shape)), dtype=np.int64).reshape(tuple(shape))
    t = np.asarray(idx if transform is None else transform(idx))
    red = set(int(a) % t.ndim for a in reduction_axes) if t.ndim else set()
    kept = [a for a in range(t.ndim) if a not in red]
    out_shape = tuple(t.shape[a] for a in kept)
    n_out = int(np.prod(out_shape)) if out_shape else 1
    moved = np.moveaxis(t, kept, list(range(len(kept)))).reshape(n_out, -1)
    return out_shape, [row.astype(np.int32) for row in moved]
