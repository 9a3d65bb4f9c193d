"""Histogram edge parameters (host side, setup-time).

Mirrors ``TOAEdges``/``make_edges`` (SRC/parameter_models.py:82-105, 290-295):
``linspace`` or ``geomspace`` of ``num_bins + 1`` values in the edge unit, then
converted to the event unit (ns) with one float64 multiply as ``bins.to(unit=
event_unit)`` does (SRC/workflows/detector_view/providers.py:205-207).  The
engine receives these float64 values bit-for-bit and derives its integer
thresholds from them, so TOA values exactly on an edge fall where scipp puts
them.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# SRC/parameter_models.py:26 -- one 14 Hz pulse period in ms, rounded up
ESS_PULSE_PERIOD_MS = float(np.ceil(1000.0 / 14 * 100) / 100)

TIME_UNIT_TO_NS = {'ns': 1.0, 'us': 1e3, 'μs': 1e3, 'ms': 1e6, 's': 1e9}


@dataclass(frozen=True)
class TOAEdges:
    """Time-of-arrival edges (defaults: 0..71.43 ms, 100 linear bins)."""

    start: float = 0.0
    stop: float = ESS_PULSE_PERIOD_MS
    num_bins: int = 100
    unit: str = 'ms'
    scale: str = 'linear'

    def __post_init__(self) -> None:
        if self.stop <= self.start:
            raise ValueError('stop must be greater than start')
        if not 1 <= self.num_bins <= 10000:
            raise ValueError('num_bins must be in [1, 10000]')
        if self.scale == 'log' and self.start <= 0:
            raise ValueError("start must be positive when scale is 'log'")
        if self.unit not in TIME_UNIT_TO_NS:
            raise ValueError(f'unsupported time unit {self.unit!r}')
        if self.scale not in ('linear', 'log'):
            raise ValueError(f'unknown scale {self.scale!r}')

    def get_edges(self) -> np.ndarray:
        """Edges in ``unit`` (``make_edges``)."""
        op = np.linspace if self.scale == 'linear' else np.geomspace
        return op(self.start, self.stop, self.num_bins + 1)

    def edges_ns(self) -> np.ndarray:
        return convert_time(self.get_edges(), self.unit, 'ns')


# SRC/parameter_models.py:118-122 (WavelengthUnit); factors to angstrom
WAVELENGTH_UNIT_TO_ANGSTROM = {'Å': 1.0, 'angstrom': 1.0, 'nm': 10.0}


@dataclass(frozen=True)
class WavelengthEdges:
    """Wavelength edges (``WavelengthEdges``, SRC/parameter_models.py:201-210;
    ``EdgesModel`` defaults 1..10, 100 linear bins, :82-105)."""

    start: float = 1.0
    stop: float = 10.0
    num_bins: int = 100
    unit: str = 'Å'
    scale: str = 'linear'

    def __post_init__(self) -> None:
        if self.stop <= self.start:
            raise ValueError('stop must be greater than start')
        if not 1 <= self.num_bins <= 10000:
            raise ValueError('num_bins must be in [1, 10000]')
        if self.scale == 'log' and self.start <= 0:
            raise ValueError("start must be positive when scale is 'log'")
        if self.unit not in WAVELENGTH_UNIT_TO_ANGSTROM:
            raise ValueError(f'unsupported wavelength unit {self.unit!r}')
        if self.scale not in ('linear', 'log'):
            raise ValueError(f'unknown scale {self.scale!r}')

    def get_edges(self) -> np.ndarray:
        op = np.linspace if self.scale == 'linear' else np.geomspace
        return op(self.start, self.stop, self.num_bins + 1)

    def edges_in(self, unit: str) -> np.ndarray:
        """Edges converted to ``unit`` (one float64 multiply, as ``bins.to``)."""
        return convert_wavelength(self.get_edges(), self.unit, unit)


def convert_wavelength(values: np.ndarray, unit: str, to: str) -> np.ndarray:
    """Wavelength unit conversion as one float64 multiply."""
    values = np.asarray(values, dtype=np.float64)
    f = WAVELENGTH_UNIT_TO_ANGSTROM[unit] / WAVELENGTH_UNIT_TO_ANGSTROM[to]
    return values if f == 1.0 else values * f


def convert_time(values: np.ndarray, unit: str, to: str) -> np.ndarray:
    """Unit conversion as one float64 multiply by the conversion factor."""
    values = np.asarray(values, dtype=np.float64)
    factor = TIME_UNIT_TO_NS[unit] / TIME_UNIT_TO_NS[to]
    return values if factor == 1.0 else values * factor


def label_slice(edges: np.ndarray, low: float, high: float) -> tuple[int, int]:
    """Bins selected by label slicing ``hist[dim, low:high]`` on bin edges:
    from the bin containing ``low`` up to the last bin overlapping
    ``[low, high)`` (SRC/workflows/monitor_workflow.py:154-167,
    SRC/workflows/detector_view/providers.py:266-270)."""
    nb = len(edges) - 1
    begin = int(np.searchsorted(edges, low, side='right')) - 1
    end = int(np.searchsorted(edges, high, side='left'))
    begin = min(max(begin, 0), nb)
    end = min(max(end, begin), nb)
    return begin, end
