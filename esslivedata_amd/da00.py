"""da00 output encoding of the finalize outputs.

The reference publishes every workflow output as an ess-streaming-data-types
``da00`` flatbuffer: ``Da00Serializer._encode`` (SRC/kafka/sink_serializers.py:
75-89) calls ``serialise_da00(source_name, timestamp_ns, scipp_to_da00(da))``,
and ``scipp_to_da00`` (SRC/kafka/scipp_da00_compat.py:22-44, 102-125) turns a
DataArray into a list of variables: the signal (``name='signal'``, the
DataArray name as ``label``), ``errors`` when there are variances, then every
coord whose values are plain arrays; datetime64 coords travel as the
timedelta since the epoch with unit ``datetime64[<unit>]``.
``da00_to_scipp`` (:47-72) is the inverse.

ess-streaming-data-types 0.27.0 and the flatbuffers runtime are not installed
(SURVEY 8(c)), so the flatbuffer is written and read here from the published
schema (``dataarray_da00.fbs``, file identifier ``da00``)::

    enum da00_dtype : byte { none, int8, uint8, int16, uint16, int32, uint32,
                             int64, uint64, float32, float64, c_string }
    table da00_Variable { name: string (required); unit: string;
        label: string; source: string; data_type: da00_dtype;
        axes: [string]; shape: [int64]; data: [ubyte] (required); }
    table da00_DataArray { source_name: string (required); timestamp: int64;
        data: [da00_Variable] (required); }
    root_type da00_DataArray;

Wire parity is unpinned (no serialized da00 payload exists offline); the
reader below is checked against the writer and against hand-laid payloads in
tests/test_da00.py.  Host code: one encode per output per finalize (1 Hz).
"""

from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Sequence

import numpy as np

from .dataarray import DataArray, Variable

FILE_IDENTIFIER = b'da00'
DTYPES = ['none', 'int8', 'uint8', 'int16', 'uint16', 'int32', 'uint32', 'int64', 'uint64',
          'float32', 'float64', 'c_string']
_NP = {n: np.dtype(n) for n in DTYPES[1:11]}
# scipp supports bool, f32, f64, i32, i64, string, datetime64: others widen on
# decode (scipp_da00_compat.py:12-19)
_DECODE_MAP = {np.dtype('uint8'): np.int32, np.dtype('int8'): np.int32,
               np.dtype('uint16'): np.int32, np.dtype('int16'): np.int32,
               np.dtype('uint32'): np.int64, np.dtype('uint64'): np.float64}


@dataclass
class Da00Variable:
    """``dataarray_da00.Variable``."""

    name: str
    data: np.ndarray
    axes: list[str]
    shape: tuple[int, ...]
    unit: str | None = None
    label: str | None = None
    source: str | None = None


# ---------------------------------------------------------------------------
# DataArray <-> variables (scipp_da00_compat.py)
# ---------------------------------------------------------------------------
def _to_variable(name: str, values, dims, unit, label=None) -> Da00Variable:
    a = np.asarray(values)
    if a.dtype.kind == 'M':  # datetime64: timedelta since the epoch
        u = np.datetime_data(a.dtype)[0]
        return Da00Variable(name, a.astype(np.int64), list(dims), tuple(a.shape),
                            f'datetime64[{u}]', label)
    return Da00Variable(name, a, list(dims), tuple(a.shape), unit, label)


def dataarray_to_da00(da: DataArray, *, signal_name: str = 'signal') -> list[Da00Variable]:
    """``scipp_to_da00``: signal (label = DataArray name), then the coords."""
    out = [_to_variable(signal_name, da.values, da.dims, da.unit, label=da.name or None)]
    for name, var in da.coords.items():
        vals = np.asarray(var.values)
        if vals.dtype == object:  # vector3 etc. are not transported
            continue
        out.append(_to_variable(name, vals, var.dims, var.unit))
    return out


def da00_to_dataarray(variables: Sequence[Da00Variable], *,
                      signal_name: str = 'signal') -> DataArray:
    """``da00_to_scipp``: the signal's label restores the name; coords whose
    dims are not a subset of the signal's are dropped."""
    byname = {}
    for v in variables:
        a = np.asarray(v.data)
        if a.dtype in _DECODE_MAP:
            a = a.astype(_DECODE_MAP[a.dtype])
        a = a.reshape(v.shape)
        unit = v.unit
        if unit is not None and unit.startswith('datetime64'):
            u = unit.split('[')[1].rstrip(']')
            a = a.astype(f'datetime64[{u}]')
            unit = u
        byname[v.name] = (a, tuple(v.axes), unit, v.label)
    data, dims, unit, label = byname.pop(signal_name)
    coords = {k: Variable(d, a, u) for k, (a, d, u, _) in byname.items()
              if k != 'errors' and set(d) <= set(dims)}
    return DataArray(data, dims, unit, coords, label or '')


# ---------------------------------------------------------------------------
# flatbuffer writer
# ---------------------------------------------------------------------------
class _Writer:
    """Front-to-back flatbuffer layout: every object referenced by a uoffset
    is placed after the referencing slot, which is patched once the target's
    position is known."""

    def __init__(self) -> None:
        self.buf = bytearray()

    def pad_to(self, align: int, extra: int = 0) -> None:
        self.buf.extend(b'\0' * ((-(len(self.buf) + extra)) % align))

    def reserve(self, n: int) -> int:
        p = len(self.buf)
        self.buf.extend(b'\0' * n)
        return p

    def patch_uoffset(self, slot: int, target: int) -> None:
        self.buf[slot:slot + 4] = struct.pack('<I', target - slot)

    def string(self, slot: int, s: str) -> None:
        b = s.encode('utf-8')
        self.pad_to(4)
        p = len(self.buf)
        self.buf.extend(struct.pack('<I', len(b)) + b + b'\0')
        self.patch_uoffset(slot, p)

    def vector(self, slot: int, payload: bytes, count: int, align: int) -> None:
        # the u32 count sits right before the (aligned) elements
        self.pad_to(max(4, align), extra=4)
        p = len(self.buf)
        self.buf.extend(struct.pack('<I', count) + payload)
        self.patch_uoffset(slot, p)

    def table(self, slots: Sequence[int | None], size: int, align: int = 4) -> int:
        """vtable then the table (soffset to it); ``slots[i]`` = byte offset of
        field i inside the table or None (absent).  Returns the table start."""
        vt = struct.pack(f'<{2 + len(slots)}H', 4 + 2 * len(slots), size,
                         *[0 if s is None else s for s in slots])
        self.pad_to(2)
        vpos = len(self.buf)
        self.buf.extend(vt)
        self.pad_to(align)
        tpos = self.reserve(size)
        self.buf[tpos:tpos + 4] = struct.pack('<i', tpos - vpos)
        return tpos


def _dtype_code(a: np.ndarray) -> int:
    name = a.dtype.name
    if name not in _NP:
        raise ValueError(f'da00 cannot carry dtype {a.dtype}')
    return DTYPES.index(name)


def serialise_da00(source_name: str, timestamp_ns: int,
                   data: Sequence[Da00Variable]) -> bytes:
    """``dataarray_da00.serialise_da00``."""
    w = _Writer()
    w.reserve(4)
    w.buf.extend(FILE_IDENTIFIER)
    # DataArray: soffset | source_name | data | pad | timestamp (8-aligned)
    root = w.table([4, 16, 8], 24, align=8)
    w.buf[0:4] = struct.pack('<I', root)
    w.buf[root + 16:root + 24] = struct.pack('<q', int(timestamp_ns))
    w.string(root + 4, source_name)
    w.pad_to(4, extra=4)
    vec = len(w.buf)
    w.buf.extend(struct.pack('<I', len(data)))
    elems = w.reserve(4 * len(data))
    w.patch_uoffset(root + 8, vec)
    for i, v in enumerate(data):
        a = np.ascontiguousarray(np.asarray(v.data))
        if a.dtype.byteorder == '>':
            a = a.astype(a.dtype.newbyteorder('<'))
        if int(np.prod(v.shape)) != a.size:
            raise ValueError(f'variable {v.name!r}: shape {v.shape} does not hold {a.size} values')
        # Variable: soffset | name unit label source axes shape data | data_type
        slots = [4, None if v.unit is None else 8, None if v.label is None else 12,
                 None if v.source is None else 16, 32, 20, 24, 28]
        t = w.table(slots, 36)
        w.patch_uoffset(elems + 4 * i, t)
        w.buf[t + 32] = _dtype_code(a)
        w.string(t + 4, v.name)
        for slot, s in ((8, v.unit), (12, v.label), (16, v.source)):
            if s is not None:
                w.string(t + slot, s)
        # axes: vector of string offsets, strings after it
        w.pad_to(4, extra=4)
        av = len(w.buf)
        w.buf.extend(struct.pack('<I', len(v.axes)))
        aslots = w.reserve(4 * len(v.axes))
        w.patch_uoffset(t + 20, av)
        for k, ax in enumerate(v.axes):
            w.string(aslots + 4 * k, ax)
        w.vector(t + 24, np.asarray(v.shape, dtype='<i8').tobytes(), len(v.shape), 8)
        w.vector(t + 28, a.tobytes(), a.nbytes, 8)
    return bytes(w.buf)


# ---------------------------------------------------------------------------
# flatbuffer reader (bounds-checked)
# ---------------------------------------------------------------------------
class _Reader:
    def __init__(self, buf) -> None:
        self.b = memoryview(bytes(buf))
        self.n = len(self.b)

    def _need(self, pos: int, size: int) -> None:
        if pos < 0 or size < 0 or pos + size > self.n:
            raise ValueError('da00: offset out of bounds')

    def u32(self, pos: int) -> int:
        self._need(pos, 4)
        return struct.unpack_from('<I', self.b, pos)[0]

    def field(self, table: int, i: int) -> int | None:
        """Absolute position of field i of the table, or None if absent."""
        self._need(table, 4)
        vt = table - struct.unpack_from('<i', self.b, table)[0]
        self._need(vt, 4)
        vt_size, t_size = struct.unpack_from('<HH', self.b, vt)
        if vt_size < 4 or vt_size % 2:
            raise ValueError('da00: bad vtable')
        self._need(vt, vt_size)
        self._need(table, t_size)
        if 4 + 2 * i >= vt_size:
            return None
        off = struct.unpack_from('<H', self.b, vt + 4 + 2 * i)[0]
        if off == 0:
            return None
        if off >= t_size:
            raise ValueError('da00: field outside its table')
        return table + off

    def deref(self, pos: int) -> int:
        return pos + self.u32(pos)

    def string(self, pos: int) -> str:
        s = self.deref(pos)
        n = self.u32(s)
        self._need(s + 4, n)
        return bytes(self.b[s + 4:s + 4 + n]).decode('utf-8')

    def vector(self, pos: int, itemsize: int) -> tuple[int, int]:
        v = self.deref(pos)
        n = self.u32(v)
        self._need(v + 4, n * itemsize)
        return v + 4, n


def deserialise_da00(buf) -> tuple[str, int, list[Da00Variable]]:
    """``dataarray_da00.deserialise_da00``: (source_name, timestamp_ns, variables).
    Malformed payloads raise ``ValueError``."""
    r = _Reader(buf)
    if r.n < 8 or bytes(r.b[4:8]) != FILE_IDENTIFIER:
        raise ValueError('not a da00 payload')
    root = r.u32(0)
    f = r.field(root, 0)
    if f is None:
        raise ValueError('da00: source_name is required')
    source = r.string(f)
    f = r.field(root, 1)
    ts = 0
    if f is not None:
        r._need(f, 8)
        ts = struct.unpack_from('<q', r.b, f)[0]
    f = r.field(root, 2)
    if f is None:
        raise ValueError('da00: data is required')
    elems, count = r.vector(f, 4)
    out = []
    for i in range(count):
        t = r.deref(elems + 4 * i)
        fn = r.field(t, 0)
        if fn is None:
            raise ValueError('da00: variable name is required')
        strs = [None if (p := r.field(t, k)) is None else r.string(p) for k in (1, 2, 3)]
        p = r.field(t, 4)
        code = r.b[p] if p is not None else 0
        if code >= len(DTYPES):
            raise ValueError(f'da00: unknown data_type {code}')
        axes = []
        if (p := r.field(t, 5)) is not None:
            a0, na = r.vector(p, 4)
            axes = [r.string(a0 + 4 * k) for k in range(na)]
        shape: tuple[int, ...] = ()
        if (p := r.field(t, 6)) is not None:
            s0, ns = r.vector(p, 8)
            shape = tuple(int(x) for x in np.frombuffer(r.b, dtype='<i8', count=ns, offset=s0))
        p = r.field(t, 7)
        if p is None:
            raise ValueError('da00: variable data is required')
        d0, nb = r.vector(p, 1)
        name = DTYPES[code]
        if name in ('none', 'c_string'):
            data = np.frombuffer(r.b, dtype=np.uint8, count=nb, offset=d0).copy()
        else:
            dt = _NP[name].newbyteorder('<')
            if nb % dt.itemsize:
                raise ValueError('da00: data size is not a multiple of the item size')
            data = np.frombuffer(r.b, dtype=dt, count=nb // dt.itemsize, offset=d0).copy()
            if int(np.prod(shape)) != data.size:
                raise ValueError('da00: shape does not match the data')
        out.append(Da00Variable(r.string(fn), data, axes, shape, *strs))
    return source, ts, out


class Da00Serializer:
    """``Da00Serializer`` (SRC/kafka/sink_serializers.py:75-89) minus the topic
    routing: payload of one finalize output."""

    def serialize(self, source_name: str, timestamp_ns: int, da: DataArray) -> bytes:
        return serialise_da00(source_name, timestamp_ns, dataarray_to_da00(da))
