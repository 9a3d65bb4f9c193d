"""ev44 event messages: native in-place decode and the reference's adapters.

Mirrors the event-message entry of the reference's Kafka boundary:

* ``deserialise_ev44`` / ``EventData`` -- ess-streaming-data-types 0.27.0
  ``eventdata_ev44`` (not vendored in the reference; pinned in
  ``requirements/base.txt``), decoded by ``lde_ev44_decode`` in the engine
  library with bounds checks, returning zero-copy numpy views into the
  payload like the reference's ``*AsNumpy`` accessors.
* ``KafkaToEv44Adapter`` (SRC/kafka/message_adapter.py:192-204),
  ``KafkaToMonitorEventsAdapter`` (:356-409), ``Ev44ToDetectorEventsAdapter``
  (:412-437), ``AdaptingMessageSource`` containment (:560-610) and
  ``FakeKafkaMessage`` (:66-96), with the same timestamp fallback, stream
  lookup (``UnmappedStreamError``) and error behaviour.
* ``serialise_ev44`` writes the flatbuffer (fake producers, tests, bench);
  the schema restatement is documented in ``csrc/lde_ev44.cpp``.

The fused native path ``BinningEngine.stage_ev44`` decodes and stages a
payload in one call without creating Python objects per message.
"""

from __future__ import annotations

import ctypes
import logging
from dataclasses import dataclass, replace
from typing import Any, Mapping, NamedTuple, Sequence

import numpy as np

from ._native import check, lib
from .preprocessors import DetectorEvents, MonitorEvents, StreamId, StreamKind, Timestamp

FILE_IDENTIFIER = b'ev44'

logger = logging.getLogger(__name__)

HAS_SOURCE_NAME = 1 << 0
HAS_MESSAGE_ID = 1 << 1
HAS_REFERENCE_TIME = 1 << 2
HAS_REFERENCE_TIME_INDEX = 1 << 3
HAS_TIME_OF_FLIGHT = 1 << 4
HAS_PIXEL_ID = 1 << 5

EV44_SINGLE_PULSE = 1
EV44_MONITOR = 2


class Ev44View(ctypes.Structure):
    """``lde_ev44_view`` (include/lde.h)."""

    _fields_ = [
        ('source_name', ctypes.c_void_p),
        ('source_name_len', ctypes.c_int64),
        ('message_id', ctypes.c_int64),
        ('reference_time', ctypes.c_void_p),
        ('n_reference_time', ctypes.c_int64),
        ('reference_time_index', ctypes.c_void_p),
        ('n_reference_time_index', ctypes.c_int64),
        ('time_of_flight', ctypes.c_void_p),
        ('n_time_of_flight', ctypes.c_int64),
        ('pixel_id', ctypes.c_void_p),
        ('n_pixel_id', ctypes.c_int64),
        ('present', ctypes.c_uint32),
    ]


class EventData(NamedTuple):
    """Field-for-field mirror of ``eventdata_ev44.EventData``.

    Absent vectors are ``None`` here (the flatbuffers accessors return a
    scalar 0, which the reference's adapters then fail on).
    """

    source_name: str | None
    message_id: int
    reference_time: np.ndarray | None
    reference_time_index: np.ndarray | None
    time_of_flight: np.ndarray | None
    pixel_id: np.ndarray | None


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return buf.view(np.uint8).reshape(-1)
    return np.frombuffer(buf, dtype=np.uint8)


def decode_view(buf) -> tuple[np.ndarray, Ev44View]:
    """Run ``lde_ev44_decode``; returns the byte array and the raw view."""
    raw = _as_u8(buf)
    view = Ev44View()
    ptr = raw.ctypes.data if raw.size else None
    check(lib().lde_ev44_decode(ptr, raw.size, ctypes.byref(view)))
    return raw, view


def _slice(raw: np.ndarray, ptr: int | None, count: int, dtype) -> np.ndarray:
    itemsize = np.dtype(dtype).itemsize
    if count == 0 or ptr is None:
        return np.empty(0, dtype=dtype)
    off = ptr - raw.ctypes.data
    return raw[off : off + count * itemsize].view(dtype)


def deserialise_ev44(buf) -> EventData:
    """Decode an ev44 payload (zero-copy views into ``buf``).

    Raises ``ValueError`` for payloads that are not well-formed ev44 (wrong
    schema identifier, truncated, offsets out of range).
    """
    raw, v = decode_view(buf)
    p = v.present
    name = None
    if p & HAS_SOURCE_NAME:
        name = bytes(_slice(raw, v.source_name, v.source_name_len, np.uint8)).decode('utf-8')
    return EventData(
        source_name=name,
        message_id=int(v.message_id),
        reference_time=_slice(raw, v.reference_time, v.n_reference_time, '<i8')
        if p & HAS_REFERENCE_TIME else None,
        reference_time_index=_slice(raw, v.reference_time_index, v.n_reference_time_index, '<i4')
        if p & HAS_REFERENCE_TIME_INDEX else None,
        time_of_flight=_slice(raw, v.time_of_flight, v.n_time_of_flight, '<i4')
        if p & HAS_TIME_OF_FLIGHT else None,
        pixel_id=_slice(raw, v.pixel_id, v.n_pixel_id, '<i4') if p & HAS_PIXEL_ID else None,
    )


# ---------------------------------------------------------------------------
# writer (flatbuffer layout: root offset, identifier, vtable, table, payloads)

def serialise_ev44(
    source_name: str,
    message_id: int,
    reference_time,
    reference_time_index,
    time_of_flight,
    pixel_id,
    *,
    omit: Sequence[str] = (),
) -> bytes:
    """Serialize an ev44 message (``eventdata_ev44.serialise_ev44`` signature).

    ``reference_time_index`` may be an int (as the reference's fakes pass it)
    or a sequence.  ``omit`` leaves the named fields out of the table, as
    other producers may (hostile-wire payloads).
    """
    if np.isscalar(reference_time_index):
        reference_time_index = [reference_time_index]
    fields = [
        ('source_name', 'str', source_name.encode('utf-8')),
        ('message_id', 'i8', int(message_id)),
        ('reference_time', 'vec', np.ascontiguousarray(reference_time, dtype='<i8')),
        ('reference_time_index', 'vec', np.ascontiguousarray(reference_time_index, dtype='<i4')),
        ('time_of_flight', 'vec', np.ascontiguousarray(time_of_flight, dtype='<i4')),
        ('pixel_id', 'vec', np.ascontiguousarray(pixel_id, dtype='<i4')),
    ]
    unknown = set(omit) - {f[0] for f in fields}
    if unknown:
        raise ValueError(f'unknown ev44 fields {sorted(unknown)}')
    # vtable at 8 (after root offset + identifier), table right after it
    n_fields = len(fields)
    vt_pos = 8
    vt_size = 4 + 2 * n_fields
    table_pos = (vt_pos + vt_size + 7) & ~7
    # table: soffset | source_name | pad | message_id (8-aligned) | 4 vector offsets
    slot = {'source_name': 4, 'message_id': 8, 'reference_time': 16,
            'reference_time_index': 20, 'time_of_flight': 24, 'pixel_id': 28}
    table_size = 32
    out = bytearray(table_pos + table_size)
    out[0:4] = np.uint32(table_pos).tobytes()
    out[4:8] = FILE_IDENTIFIER
    vt = [vt_size, table_size] + [0] * n_fields
    out[table_pos : table_pos + 4] = np.int32(table_pos - vt_pos).tobytes()
    for i, (name, kind, value) in enumerate(fields):
        if name in omit:
            continue
        vt[2 + i] = slot[name]
        fpos = table_pos + slot[name]
        if kind == 'i8':
            out[fpos : fpos + 8] = np.int64(value).tobytes()
            continue
        if kind == 'str':
            payload, count, align = value + b'\0', len(value), 4
        else:
            payload, count, align = value.tobytes(), value.size, max(4, value.itemsize)
        # element data aligned to its size: the u32 count sits just before it
        start = len(out) + 4
        start = (start + align - 1) // align * align
        out.extend(b'\0' * (start - 4 - len(out)))
        cpos = len(out)
        out.extend(np.uint32(count).tobytes())
        out.extend(payload)
        out.extend(b'\0' * (-len(out) % 4))
        out[fpos : fpos + 4] = np.uint32(cpos - fpos).tobytes()
    out[vt_pos : vt_pos + vt_size] = np.asarray(vt, dtype='<u2').tobytes()
    return bytes(out)


# ---------------------------------------------------------------------------
# adapters (SRC/kafka/message_adapter.py)


class UnmappedStreamError(Exception):
    """A (topic, source_name) pair with no entry in the stream LUT."""


@dataclass(frozen=True)
class InputStreamKey:
    topic: str
    source_name: str


@dataclass(frozen=True)
class Message:
    timestamp: Timestamp
    stream: StreamId
    value: Any


class FakeKafkaMessage:
    """message_adapter.py:66-96."""

    def __init__(self, *, key: bytes = b'', value: bytes, topic: str, timestamp: int = 0,
                 timestamp_type: int = 0) -> None:
        self._key, self._value, self._topic = key, value, topic
        self._timestamp, self._timestamp_type = timestamp, timestamp_type

    def error(self) -> Any | None:
        return None

    def key(self) -> bytes:
        return self._key

    def value(self) -> bytes:
        return self._value

    def timestamp(self) -> tuple[int, int]:
        return (self._timestamp_type, self._timestamp)

    def topic(self) -> str:
        return self._topic


class _KafkaAdapter:
    def __init__(self, *, stream_lut: Mapping[InputStreamKey, str] | None = None,
                 stream_kind: StreamKind) -> None:
        self._stream_lut = stream_lut
        self._stream_kind = stream_kind

    def get_stream_id(self, topic: str, source_name: str) -> StreamId:
        """message_adapter.py:158-173."""
        if self._stream_lut is None:
            return StreamId(kind=self._stream_kind, name=source_name)
        try:
            resolved = self._stream_lut[InputStreamKey(topic=topic, source_name=source_name)]
        except KeyError:
            raise UnmappedStreamError(source_name) from None
        return StreamId(kind=self._stream_kind, name=resolved)


def _timestamp(reference_time: np.ndarray, message) -> Timestamp:
    # message_adapter.py:197-201 (a fallback for reused serialized test data)
    if reference_time.size > 0:
        return Timestamp.from_ns(int(reference_time[-1]))
    return Timestamp.from_ns(int(message.timestamp()[1]) * 1_000_000)


def _require(value, what: str):
    if value is None:
        # the reference fails here on the flatbuffers scalar-0 default
        raise ValueError(f'ev44: {what} is absent')
    return value


class KafkaToEv44Adapter(_KafkaAdapter):
    """message_adapter.py:192-204: ev44 payload -> ``Message[EventData]``."""

    schema = 'ev44'

    def __init__(self, *, stream_lut=None, stream_kind: StreamKind = StreamKind.DETECTOR_EVENTS):
        super().__init__(stream_lut=stream_lut, stream_kind=stream_kind)

    def adapt(self, message) -> Message:
        ev44 = deserialise_ev44(message.value())
        name = _require(ev44.source_name, 'source_name')
        stream = self.get_stream_id(topic=message.topic(), source_name=name)
        ts = _timestamp(_require(ev44.reference_time, 'reference_time'), message)
        return Message(timestamp=ts, stream=stream, value=ev44)


class Ev44ToDetectorEventsAdapter:
    """message_adapter.py:412-437: ``EventData`` -> ``DetectorEvents``."""

    def __init__(self, *, merge_detectors: bool = False) -> None:
        self._merge_detectors = merge_detectors

    def adapt(self, message: Message) -> Message:
        stream = message.stream
        if self._merge_detectors:
            stream = replace(stream, name='unified_detector')
        ev44 = message.value
        _require(ev44.reference_time_index, 'reference_time_index')
        _require(ev44.time_of_flight, 'time_of_flight')
        _require(ev44.pixel_id, 'pixel_id')
        return Message(timestamp=message.timestamp, stream=stream,
                       value=DetectorEvents.from_ev44(ev44))


class KafkaToMonitorEventsAdapter(_KafkaAdapter):
    """message_adapter.py:356-409: ev44 -> ``MonitorEvents`` (or
    ``DetectorEvents`` for pixellated monitors), without the single-pulse
    check and ignoring ``pixel_id`` for plain monitors."""

    schema = 'ev44'

    def __init__(self, stream_lut=None, *, pixellated_sources: frozenset[str] = frozenset()):
        super().__init__(stream_lut=stream_lut, stream_kind=StreamKind.MONITOR_EVENTS)
        self._pixellated_sources = pixellated_sources

    def adapt(self, message) -> Message:
        ev44 = deserialise_ev44(message.value())
        name = _require(ev44.source_name, 'source_name')
        stream = self.get_stream_id(topic=message.topic(), source_name=name)
        ts = _timestamp(_require(ev44.reference_time, 'reference_time'), message)
        toa = _require(ev44.time_of_flight, 'time_of_flight')
        if stream.name in self._pixellated_sources:
            value: MonitorEvents = DetectorEvents(
                pixel_id=_require(ev44.pixel_id, 'pixel_id'), time_of_arrival=toa, unit='ns')
        else:
            value = MonitorEvents(time_of_arrival=toa, unit='ns')
        return Message(timestamp=ts, stream=stream, value=value)


class ChainedAdapter:
    """Two adapters applied in sequence (message_adapter.py ChainedAdapter)."""

    def __init__(self, first, second) -> None:
        self._first, self._second = first, second

    def adapt(self, message):
        return self._second.adapt(self._first.adapt(message))


class AdaptingMessageSource:
    """Per-message containment: a payload that cannot be adapted is dropped
    (logged), later messages are unaffected (message_adapter.py:560-610)."""

    def __init__(self, source, adapter, *, raise_on_error: bool = False) -> None:
        self._source, self._adapter = source, adapter
        self._raise_on_error = raise_on_error

    def get_messages(self) -> list:
        adapted = []
        for msg in self._source.get_messages():
            try:
                adapted.append(self._adapter.adapt(msg))
            except UnmappedStreamError:
                if self._raise_on_error:
                    raise
            except Exception:
                logger.exception('Error adapting message from topic %s', msg.topic())
                if self._raise_on_error:
                    raise
        return adapted
