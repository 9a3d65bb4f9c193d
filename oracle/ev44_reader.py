"""TEST INFRASTRUCTURE ONLY -- CPU checker for the native ev44 decoder.

Only tests/ may import this module; the product path (esslivedata_amd) never
does.  It restates, in plain Python, how the reference reads an ev44 payload:

* flatbuffers 25.12.19 Python runtime (``flatbuffers/table.py``):
  ``Table.Offset`` (vtable lookup: vtable = pos - soffset; a slot beyond the
  vtable size, or 0, means absent), ``Indirect`` (pos + uoffset),
  ``String`` / ``VectorLen`` / ``Vector`` (u32 count before the data);
* ess-streaming-data-types 0.27.0 generated ``Event44Message`` accessors
  (slots 4, 6, 8, 10, 12, 14 = source_name, message_id, reference_time,
  reference_time_index, time_of_flight, pixel_id) and
  ``check_schema_identifier`` (bytes 4:8 must be b"ev44");
* adapter rules of SRC/kafka/message_adapter.py:192-204, 380-409 and
  SRC/preprocessors/to_nxevent_data.py:16-19, 57-62.

Neither library is vendored under /root/reference nor installed here, and the
reference's tests hold no serialized ev44 bytes (they build payloads with
``serialise_ev44`` at run time, tests/helpers/hostile_wire.py:52-133), so the
byte layout is **parity unpinned**: this reader and the C decoder are two
independent restatements of the published format, checked against each other
and against the reference's hostile-wire behaviour.

Out-of-range reads raise (``struct.error`` / ``ValueError``) as the Python
runtime does; absent vectors are ``None`` (the runtime returns scalar 0).
"""

from __future__ import annotations

import struct

import numpy as np

SLOTS = {
    'source_name': 4,
    'message_id': 6,
    'reference_time': 8,
    'reference_time_index': 10,
    'time_of_flight': 12,
    'pixel_id': 14,
}


class WrongSchema(ValueError):
    pass


def _u32(b: bytes, pos: int) -> int:
    if pos < 0:
        raise struct.error('negative offset')
    return struct.unpack_from('<I', b, pos)[0]


def _field_offset(b: bytes, table: int, slot: int) -> int:
    vtable = table - struct.unpack_from('<i', b, table)[0]
    if vtable < 0:
        raise struct.error('negative vtable')
    vt_size = struct.unpack_from('<H', b, vtable)[0]
    if slot < vt_size:
        return struct.unpack_from('<H', b, vtable + slot)[0]
    return 0


def _vector(b: bytes, table: int, slot: int, dtype):
    off = _field_offset(b, table, slot)
    if off == 0:
        return None
    pos = table + off
    start = pos + _u32(b, pos)
    n = _u32(b, start)
    return np.frombuffer(b, dtype=dtype, count=n, offset=start + 4)


def read_ev44(payload: bytes) -> dict:
    b = bytes(payload)
    if len(b) < 8 or b[4:8] != b'ev44':
        raise WrongSchema(f'wrong schema identifier {b[4:8]!r}')
    table = _u32(b, 0)
    out = {}
    off = _field_offset(b, table, SLOTS['source_name'])
    if off:
        pos = table + off
        start = pos + _u32(b, pos)
        n = _u32(b, start)
        if start + 4 + n > len(b):
            raise struct.error('string out of range')
        out['source_name'] = b[start + 4 : start + 4 + n].decode('utf-8')
    else:
        out['source_name'] = None
    off = _field_offset(b, table, SLOTS['message_id'])
    out['message_id'] = struct.unpack_from('<q', b, table + off)[0] if off else 0
    out['reference_time'] = _vector(b, table, SLOTS['reference_time'], '<i8')
    out['reference_time_index'] = _vector(b, table, SLOTS['reference_time_index'], '<i4')
    out['time_of_flight'] = _vector(b, table, SLOTS['time_of_flight'], '<i4')
    out['pixel_id'] = _vector(b, table, SLOTS['pixel_id'], '<i4')
    return out


def adapt_timestamp_ns(ev: dict, kafka_timestamp_ms: int) -> int:
    """message_adapter.py:197-201 (reference_time[-1], else Kafka ms)."""
    rt = ev['reference_time']
    if rt is None:
        raise AttributeError("'int' object has no attribute 'size'")
    return int(rt[-1]) if rt.size > 0 else int(kafka_timestamp_ms) * 1_000_000


def require_single_pulse(ev: dict) -> None:
    """to_nxevent_data.py:16-19."""
    index = ev['reference_time_index']
    if len(index) > 1 or index[0] != 0 or len(ev['reference_time']) > 1:
        raise NotImplementedError('Processing multi-pulse messages is not supported.')
