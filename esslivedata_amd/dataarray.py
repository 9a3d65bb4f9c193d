"""Minimal labelled-array container for workflow outputs.

The reference returns ``scipp.DataArray`` outputs that downstream code only
serialises to da00 (SRC/kafka/sink_serializers.py:75-89).  scipp is not part
of this image, so outputs use this small stand-in with the same information:
dims, values (numpy), unit and named coords.  ``to_scipp()`` converts when
scipp is importable.
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
            new[k] = v if isinstance(v, Variable) else Variable((), v)
        return DataArray(self.values, self.dims, self.unit, new, self.name)

    def to_scipp(self):  # pragma: no cover - scipp absent in this image
        import scipp as sc

        coords = {
            k: sc.array(dims=list(v.dims), values=v.values, unit=v.unit)
            if v.dims
            else sc.scalar(v.values, unit=v.unit)
            for k, v in self.coords.items()
        }
        data = (
            sc.array(dims=list(self.dims), values=self.values, unit=self.unit)
            if self.dims
            else sc.scalar(self.value, unit=self.unit)
        )
        return sc.DataArray(data, coords=coords)
