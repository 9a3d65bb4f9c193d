"""Wavelength-mode inputs (setup time, host side).

The reference's detector view in ``'wavelength'`` mode histograms each event's
wavelength instead of its time of arrival (SRC/workflows/detector_view/
factory.py:134-169, providers.py:77-95).  The wavelength comes from
essreduce's ``GenericUnwrapWorkflow``: a lookup table over (flight-path
distance ``Ltotal``, event time offset) read from ``LookupTableFilename`` and
interpolated per event, with ``Ltotal`` from the detector geometry (the
factory refuses wavelength mode without geometry, factory.py:137-142).

essreduce is not part of /root/reference and its table files are not in the
image, so the table arrives here as arrays on a regular grid, and the per-event
lookup is the bilinear form the engine documents (include/lde.h,
``lde_set_coord_lut``).  Per-event work runs on the GPU (lde_coord.hip);
this module only computes the per-pixel distances and validates the grid.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# h / m_n in m * angstrom / s: lambda[A] = H_OVER_MN * t[s] / L[m]
H_OVER_MN = 3956.0339


@dataclass(frozen=True)
class WavelengthLookupTable:
    """Coordinate table on a regular (distance, time) grid.

    ``table[i, j]`` is the wavelength (in ``unit``) at distance
    ``distance0 + i * distance_step`` (m) and time offset ``time0 + j *
    time_step`` (ns); NaN marks undefined regions (dropped events)."""

    table: np.ndarray
    distance0: float
    distance_step: float
    time0: float
    time_step: float
    unit: str = 'Å'

    def __post_init__(self) -> None:
        t = np.asarray(self.table, dtype=np.float64)
        if t.ndim != 2 or t.shape[0] < 2 or t.shape[1] < 2:
            raise ValueError('the table needs at least 2 x 2 grid points (distance, time)')
        if not (self.distance_step > 0 and self.time_step > 0):
            raise ValueError('grid steps must be positive')
        object.__setattr__(self, 'table', np.ascontiguousarray(t))

    @property
    def distances(self) -> np.ndarray:
        return self.distance0 + self.distance_step * np.arange(self.table.shape[0])

    @property
    def times(self) -> np.ndarray:
        return self.time0 + self.time_step * np.arange(self.table.shape[1])


def ideal_lookup_table(distance_min: float, distance_max: float, n_distance: int,
                       time_max_ns: float, n_time: int) -> WavelengthLookupTable:
    """Table of the direct-flight relation ``lambda = (h / m_n) t / L`` (no
    chopper cascade, one frame) on ``n_distance x n_time`` points from t = 0."""
    d_step = (distance_max - distance_min) / (n_distance - 1)
    t_step = time_max_ns / (n_time - 1)
    d = distance_min + d_step * np.arange(n_distance)
    t = t_step * np.arange(n_time)
    table = H_OVER_MN * (t[None, :] * 1e-9) / d[:, None]
    return WavelengthLookupTable(table, distance_min, d_step, 0.0, t_step)


def pixel_ltotal(positions: np.ndarray, *, source_position=(0.0, 0.0, -76.55),
                 sample_position=(0.0, 0.0, 0.0)) -> np.ndarray:
    """``Ltotal = |sample - source| + |position - sample|`` per pixel (m)."""
    p = np.asarray(positions, dtype=np.float64).reshape(-1, 3)
    src = np.asarray(source_position, dtype=np.float64)
    smp = np.asarray(sample_position, dtype=np.float64)
    return np.linalg.norm(smp - src) + np.linalg.norm(p - smp, axis=1)


def distance_per_pid(detector_number: np.ndarray, ltotal: np.ndarray, pid_offset: int,
                     lut_len: int) -> np.ndarray:
    """Per pixel id ``pid_offset + k`` (the engine LUT's indexing): the pixel's
    ``Ltotal``, NaN for ids that are not detector pixels."""
    dn = np.asarray(detector_number).ravel().astype(np.int64)
    lt = np.asarray(ltotal, dtype=np.float64).ravel()
    if dn.shape != lt.shape:
        raise ValueError('one Ltotal per detector pixel is required')
    out = np.full(int(lut_len), np.nan)
    k = dn - int(pid_offset)
    ok = (k >= 0) & (k < lut_len)
    out[k[ok]] = lt[ok]
    return out
