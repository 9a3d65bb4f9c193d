"""Labelled-array outputs of the workflows.

The reference returns ``scipp.DataArray`` outputs: the unchanged caller
``Job._add_time_coords`` stamps them (SRC/core/job.py:212-262) and
``Da00Serializer`` serialises them (SRC/kafka/sink_serializers.py:75-89,
``scipp_to_da00``, SRC/kafka/scipp_da00_compat.py:22-116).  The workflows
build their outputs in this small stand-in (dims, numpy values, unit, named
coords) and :func:`publish` hands them over as ``scipp.DataArray`` whenever
``import scipp`` succeeds, so both callers work unchanged; without scipp (this
image) the stand-ins are returned, with the same information.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

import numpy as np


@dataclass
class Variable:
    dims: tuple[str, ...]
    values: np.ndarray | Any
    unit: str | None = None

    @property
    def value(self):
        if self.dims:
            raise ValueError('value is only defined for 0-D variables')
        return self.values.item() if isinstance(self.values, np.ndarray) else self.values


@dataclass
class DataArray:
    values: np.ndarray
    dims: tuple[str, ...]
    unit: str | None = 'counts'
    coords: dict[str, Variable] = field(default_factory=dict)
    name: str = ''

    @property
    def sizes(self) -> dict[str, int]:
        return dict(zip(self.dims, np.shape(self.values)))

    @property
    def shape(self) -> tuple[int, ...]:
        return tuple(np.shape(self.values))

    @property
    def dtype(self):
        return np.asarray(self.values).dtype

    @property
    def value(self):
        if self.dims:
            raise ValueError('value is only defined for 0-D data')
        return np.asarray(self.values).item()

    def sum(self) -> 'DataArray':
        return DataArray(np.asarray(self.values).sum(), (), self.unit)

    def nansum(self) -> 'DataArray':
        return DataArray(np.nansum(self.values), (), self.unit)

    def assign_coords(self, **coords) -> 'DataArray':
        new = dict(self.coords)
        for k, v in coords.items():
            # variables (stand-in or scipp) are kept; plain values become 0-D
            new[k] = v if isinstance(v, Variable) or hasattr(v, 'dims') else Variable((), v)
        return DataArray(self.values, self.dims, self.unit, new, self.name)

    def to_scipp(self):
        """The same array as a ``scipp.DataArray`` (dtypes kept: float32
        BIFROST counts stay float32, the int64 'ns' time coords int64)."""
        sc = scipp_module()
        if sc is None:
            raise ImportError('scipp is not importable')
        coords = {k: _sc_variable(sc, v.dims, v.values, v.unit) if isinstance(v, Variable) else v
                  for k, v in self.coords.items()}
        return sc.DataArray(_sc_variable(sc, self.dims, self.values, self.unit), coords=coords)


# ``import scipp`` is attempted once per process: a failing import costs a
# path search, and finalize runs per batch (reset_scipp_module() re-probes)
_SCIPP: list = []


def scipp_module():
    """The scipp module, or None when it is not importable."""
    if not _SCIPP:
        try:
            import scipp
        except ImportError:
            scipp = None
        _SCIPP.append(scipp)
    return _SCIPP[0]


def reset_scipp_module() -> None:
    _SCIPP.clear()


# numpy dtypes the stand-ins carry, as scipp dtype names (counts as float64 /
# float32, exact partial sums as uint64 -> int64 is not needed: scipp has no
# unsigned 64-bit dtype, so they are refused, as are object / string arrays)
_SC_DTYPES = {'float64': 'float64', 'float32': 'float32', 'int64': 'int64', 'int32': 'int32',
              'bool': 'bool'}


def _sc_variable(sc, dims, values, unit):
    a = np.asarray(values)
    dt = _SC_DTYPES.get(str(a.dtype))
    if dt is None:
        raise TypeError(f'no scipp dtype for a {a.dtype} output (float64, float32, int64, int32, bool)')
    if not dims:
        return sc.scalar(a.item(), unit=unit, dtype=dt)
    return sc.array(dims=list(dims), values=a, unit=unit, dtype=dt)


def scalar(value, *, unit: str | None = None):
    """A 0-D variable: ``sc.scalar`` when scipp is importable, else the stand-in
    (``Timestamp.to_scipp``, SRC/core/timestamp.py:216-220)."""
    sc = scipp_module()
    if sc is not None:
        return _sc_variable(sc, (), value, unit)
    return Variable((), np.asarray(value), unit)


def publish(outputs: dict) -> dict:
    """The workflow's output dict as the reference's callers receive it:
    stand-ins converted to ``scipp.DataArray`` when scipp is importable (other
    values, e.g. a caller's own ROI request echoed back, pass unchanged)."""
    if scipp_module() is None:
        return outputs
    return {k: v.to_scipp() if isinstance(v, DataArray) else v for k, v in outputs.items()}


def add_time_coords(data: dict, start_time, end_time) -> dict:
    """``Job._add_time_coords`` (SRC/core/job.py:212-262): 0-D
    ``start_time`` / ``time`` (int64, 'ns') on every data array that carries
    neither yet -- stand-ins and ``scipp.DataArray`` alike (anything with
    ``coords`` and ``assign_coords``, as the reference stamps every
    DataArray, so outputs already published as scipp objects are stamped
    too); no time bounds -> ValueError."""
    if start_time is None or end_time is None:
        raise ValueError('Job has no time bounds to stamp on its outputs: finalized before '
                         'accumulating any primary data.')
    st, tt = start_time.to_scipp(), end_time.to_scipp()

    def stamp(v):
        if 'start_time' in v.coords or 'time' in v.coords:
            return v
        return v.assign_coords(start_time=st, time=tt)

    def stampable(v):
        return hasattr(v, 'coords') and hasattr(v, 'assign_coords')

    return {k: stamp(v) if stampable(v) else v for k, v in data.items()}
