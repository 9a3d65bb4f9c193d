"""Named-dimension pixel-index arrays for logical-view transforms.

The reference's logical views are scipp transforms of the detector data
(``fold``, ``transpose``, label slicing ``['wire', 0]``, ``flatten``) followed
by ``bins.concat(reduction_dim)`` (SRC/workflows/detector_view/
projectors.py:243-270, types.py:100-126).  The engine needs only where each
detector pixel ends up, so the same transform is applied, once at setup, to
this stand-in holding the flat pixel index of every element.  It implements
the subset of the scipp API the reference's transforms use (dummy, BIFROST,
LOKI, DREAM and MAGIC views), with scipp's rules:

* ``fold(dim, sizes)``: the dim is replaced in place by ``sizes`` (row-major,
  at most one ``-1``);
* ``transpose(dims)``: a permutation of all dims;
* ``flatten(dims, to)``: ``dims`` must be adjacent and in memory order
  (scipp raises otherwise); ``dims=None`` flattens everything;
* ``x[dim, i]`` drops ``dim``; ``x[dim, a:b]`` keeps it;
* ``to(dtype=...)`` and other value-only operations are no-ops.

Reduction over named dims is done by :func:`projection.logical_lut`.
"""

from __future__ import annotations

from typing import Mapping, Sequence

import numpy as np


class LogicalIndex:
    """Flat pixel indices with named dims (scipp ``DataArray`` stand-in)."""

    def __init__(self, values: np.ndarray, dims: Sequence[str]) -> None:
        values = np.asarray(values)
        dims = tuple(dims)
        if values.ndim != len(dims):
            raise ValueError(f'{len(dims)} dims {dims} for an array of shape {values.shape}')
        if len(set(dims)) != len(dims):
            raise ValueError(f'duplicate dims {dims}')
        self.values = values
        self.dims = dims

    # -- metadata ----------------------------------------------------------
    @property
    def dim(self) -> str:
        if len(self.dims) != 1:
            raise ValueError(f'dim is only defined for 1-D data, got dims {self.dims}')
        return self.dims[0]

    @property
    def sizes(self) -> dict[str, int]:
        return dict(zip(self.dims, self.values.shape))

    @property
    def shape(self) -> tuple[int, ...]:
        return tuple(self.values.shape)

    @property
    def ndim(self) -> int:
        return self.values.ndim

    def __array__(self, dtype=None, copy=None):
        return self.values if dtype is None else self.values.astype(dtype)

    def __repr__(self) -> str:
        return f'LogicalIndex(sizes={self.sizes})'

    # -- value-only operations (no effect on where pixels go) --------------
    def to(self, *, dtype=None, unit=None, copy=True) -> 'LogicalIndex':
        return self

    def copy(self, deep: bool = True) -> 'LogicalIndex':
        return LogicalIndex(self.values.copy(), self.dims)

    # -- structural operations ---------------------------------------------
    def _axis(self, dim: str) -> int:
        try:
            return self.dims.index(dim)
        except ValueError:
            raise KeyError(f'dim {dim!r} not in {self.dims}') from None

    def fold(self, dim: str, sizes: Mapping[str, int] | None = None, *,
             dims: Sequence[str] | None = None, shape: Sequence[int] | None = None) -> 'LogicalIndex':
        if sizes is None:
            if dims is None or shape is None:
                raise ValueError('fold needs sizes, or dims and shape')
            sizes = dict(zip(dims, shape))
        ax = self._axis(dim)
        n = self.values.shape[ax]
        new = dict(sizes)
        free = [d for d, s in new.items() if s == -1]
        if len(free) > 1:
            raise ValueError('fold: at most one size may be -1')
        known = int(np.prod([s for s in new.values() if s != -1])) if new else 1
        if free:
            if known == 0 or n % known:
                raise ValueError(f'fold: cannot fold {n} into {sizes}')
            new[free[0]] = n // known
        if int(np.prod(list(new.values()))) != n:
            raise ValueError(f'fold: sizes {sizes} do not multiply to {n}')
        out_dims = self.dims[:ax] + tuple(new) + self.dims[ax + 1:]
        out_shape = self.values.shape[:ax] + tuple(new.values()) + self.values.shape[ax + 1:]
        return LogicalIndex(self.values.reshape(out_shape), out_dims)

    def transpose(self, dims: Sequence[str] | None = None) -> 'LogicalIndex':
        if dims is None:
            dims = self.dims[::-1]
        dims = tuple(dims)
        if sorted(dims) != sorted(self.dims):
            raise ValueError(f'transpose: {dims} is not a permutation of {self.dims}')
        axes = [self._axis(d) for d in dims]
        return LogicalIndex(np.transpose(self.values, axes), dims)

    def flatten(self, dims: Sequence[str] | None = None, to: str | None = None) -> 'LogicalIndex':
        if to is None:
            raise ValueError('flatten needs a target dim name (to=...)')
        if dims is None:
            dims = self.dims
        dims = tuple(dims)
        if not dims:
            return LogicalIndex(self.values[..., None], self.dims + (to,))
        axes = [self._axis(d) for d in dims]
        if axes != list(range(axes[0], axes[0] + len(axes))):
            raise ValueError(f'flatten: dims {dims} are not adjacent and in order in {self.dims}')
        a0, a1 = axes[0], axes[-1] + 1
        shape = self.values.shape
        out_shape = shape[:a0] + (int(np.prod(shape[a0:a1])),) + shape[a1:]
        out_dims = self.dims[:a0] + (to,) + self.dims[a1:]
        # a transposed (non-contiguous) view is copied into the new memory order
        return LogicalIndex(np.ascontiguousarray(self.values).reshape(out_shape), out_dims)

    def rename_dims(self, mapping: Mapping[str, str] | None = None, **names) -> 'LogicalIndex':
        m = dict(mapping or {}, **names)
        return LogicalIndex(self.values, tuple(m.get(d, d) for d in self.dims))

    def __getitem__(self, key):
        if not (isinstance(key, tuple) and len(key) == 2 and isinstance(key[0], str)):
            return self.values[key]  # positional numpy indexing: a plain array
        dim, sel = key
        ax = self._axis(dim)
        index = [slice(None)] * self.ndim
        if isinstance(sel, slice):
            index[ax] = sel
            return LogicalIndex(self.values[tuple(index)], self.dims)
        i = int(sel)
        n = self.values.shape[ax]
        if not -n <= i < n:
            raise IndexError(f'index {i} out of range for dim {dim!r} of size {n}')
        index[ax] = i
        return LogicalIndex(self.values[tuple(index)], self.dims[:ax] + self.dims[ax + 1:])

    # plain-numpy transforms (``idx.reshape(15, 900)``, ``a.T[1:]``) keep
    # working; their results are positional arrays without dim names
    def reshape(self, *shape) -> np.ndarray:
        return self.values.reshape(*shape)

    @property
    def T(self) -> np.ndarray:
        return self.values.T


def detector_index(detector_number: np.ndarray, dims: Sequence[str] | None = None) -> LogicalIndex:
    """Index array shaped like ``detector_number`` with its dims (1-D:
    ``detector_number``, as the raw NeXus detector data has)."""
    dn = np.asarray(detector_number)
    if dims is None:
        dims = ('detector_number',) if dn.ndim == 1 else tuple(f'dim_{i}' for i in range(dn.ndim))
    return LogicalIndex(np.arange(dn.size, dtype=np.int64).reshape(dn.shape), dims)


def reduction_dims(reduction_dim: str | Sequence[str] | None) -> tuple[str, ...]:
    """``reduction_dim`` as the tuple of dims to merge (projectors.py:199-207)."""
    if reduction_dim is None:
        return ()
    if isinstance(reduction_dim, str):
        return (reduction_dim,)
    return tuple(reduction_dim)
