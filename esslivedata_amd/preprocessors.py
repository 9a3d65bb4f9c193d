"""Accumulator-protocol side of the drop-in boundary (preprocessing).

Mirrors the reference's preprocessing plugins for event streams:

* ``MonitorEvents`` / ``DetectorEvents`` (SRC/preprocessors/to_nxevent_data.py:22-69)
  with the same length check and single-pulse restriction.
* ``EventStaging`` replaces ``ToNXevent_data`` (to_nxevent_data.py:127-208) and,
  for detectors, ``GroupByPixel`` (SRC/preprocessors/group_by_pixel.py:17-57):
  it keeps the zero-copy ev44 views of one batch and hands them to the GPU
  workflow, which stages them into pinned memory and HBM.  Pixel grouping,
  projection and binning happen on the GPU, so no host-side concat or
  ``group`` copy of the events is made.  Error behaviour follows the reference:
  unit other than 'ns' -> ValueError; mixing detector and monitor events ->
  ValueError; ``get()`` before ``add()`` -> ValueError; ``get()`` while a
  previous result was not released -> RuntimeError.
* ``GpuPreprocessorFactory`` plays the role of ``DetectorPreprocessorFactory`` /
  ``ReductionPreprocessorFactory`` (SRC/preprocessors/detector_data.py:41-60,
  data_reduction.py:21-39) for event streams.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Any, ClassVar, Sequence

import numpy as np


class Timestamp:
    """Nanoseconds since the Unix epoch (mirror of SRC/core/timestamp.py:140-170)."""

    __slots__ = ('_ns',)

    def __init__(self, *, ns: int) -> None:
        self._ns = int(ns)

    @classmethod
    def from_ns(cls, ns: int) -> 'Timestamp':
        return cls(ns=int(ns))

    @classmethod
    def from_seconds(cls, seconds: float) -> 'Timestamp':
        return cls(ns=int(seconds * 1_000_000_000))

    def to_ns(self) -> int:
        return self._ns

    def to_scipp(self):
        """A 0-D int64 scalar with unit 'ns' (SRC/core/timestamp.py:216-220):
        a scipp scalar when scipp is importable, else the stand-in variable."""
        from .dataarray import scalar

        return scalar(np.int64(self._ns), unit='ns')

    def __eq__(self, other) -> bool:
        return isinstance(other, Timestamp) and other._ns == self._ns

    def __lt__(self, other: 'Timestamp') -> bool:
        return self._ns < other._ns

    def __hash__(self) -> int:
        return hash(self._ns)

    def __repr__(self) -> str:
        return f'Timestamp(ns={self._ns})'


def _require_single_pulse(ev44) -> None:
    """to_nxevent_data.py:16-19."""
    index = ev44.reference_time_index
    if len(index) > 1 or index[0] != 0 or len(ev44.reference_time) > 1:
        raise NotImplementedError('Processing multi-pulse messages is not supported.')


@dataclass
class MonitorEvents:
    time_of_arrival: Sequence[int]
    unit: str

    @staticmethod
    def from_ev44(ev44) -> 'MonitorEvents':
        _require_single_pulse(ev44)
        return MonitorEvents(time_of_arrival=ev44.time_of_flight, unit='ns')


@dataclass
class DetectorEvents(MonitorEvents):
    pixel_id: Sequence[int]

    def __post_init__(self) -> None:
        if len(self.pixel_id) != len(self.time_of_arrival):
            raise ValueError(
                f'pixel_id and time_of_arrival must have the same length, '
                f'got {len(self.pixel_id)} and {len(self.time_of_arrival)}'
            )

    @staticmethod
    def from_ev44(ev44) -> 'DetectorEvents':
        _require_single_pulse(ev44)
        return DetectorEvents(
            pixel_id=ev44.pixel_id, time_of_arrival=ev44.time_of_flight, unit='ns'
        )


@dataclass
class StagedEvents:
    """One batch of event messages, handed from the preprocessor to the GPU
    workflow (the GPU counterpart of ``ToNXevent_data.get``'s binned array)."""

    time_of_arrival: list[np.ndarray]
    pixel_id: list[np.ndarray] | None
    event_time_zero: list[int]
    unit: str = 'ns'

    @property
    def n_events(self) -> int:
        return int(sum(len(t) for t in self.time_of_arrival))

    @property
    def n_messages(self) -> int:
        return len(self.time_of_arrival)


def _int32_view(a) -> np.ndarray:
    """The message array as contiguous int32 (zero-copy when it already is).
    Wider integer arrays whose values do not all fit are kept as they are:
    the engine's ``stage`` converts them with range checks (an id beyond int32
    is an unknown id and dropped, as ``group_event_data`` drops it; it must
    not wrap onto a valid pixel)."""
    arr = np.asarray(a)
    if arr.dtype.kind not in 'iu':
        raise TypeError(f'event arrays must be integer, got {arr.dtype}')
    if arr.dtype == np.int32 or arr.size == 0 or (
            int(arr.min()) >= -(2**31) and int(arr.max()) < 2**31):
        return np.ascontiguousarray(arr, dtype=np.int32)
    return np.ascontiguousarray(arr)


class EventStaging:
    """``Accumulator[DetectorEvents | MonitorEvents, StagedEvents]``."""

    is_context: ClassVar[bool] = False

    def __init__(self, detector_number: np.ndarray | None = None) -> None:
        # detector_number is kept for GroupByPixel API parity; grouping is
        # applied on the GPU through the view's LUT
        self._detector_number = detector_number
        self._toa: list[np.ndarray] = []
        self._pid: list[np.ndarray] = []
        self._timestamps: list[int] = []
        self._have_event_id: bool | None = None
        self._buffers_in_use = False

    def add(self, timestamp: Timestamp, data: MonitorEvents) -> bool:
        if data.unit != 'ns':
            raise ValueError(f"Expected unit 'ns', got '{data.unit}'")
        is_det = isinstance(data, DetectorEvents)
        if self._have_event_id is None:
            self._have_event_id = is_det
        elif self._have_event_id != is_det:
            raise ValueError('Inconsistent event_id')
        self._timestamps.append(timestamp.to_ns())
        self._toa.append(_int32_view(data.time_of_arrival))
        if is_det:
            self._pid.append(_int32_view(data.pixel_id))
        return True

    def get(self) -> StagedEvents:
        if self._have_event_id is None:
            raise ValueError('No data has been added')
        if self._buffers_in_use:
            raise RuntimeError(
                'Buffers from a previous get() have not been released. '
                'Call release_buffers() after the result has been consumed.'
            )
        self._buffers_in_use = True
        out = StagedEvents(
            time_of_arrival=list(self._toa),
            pixel_id=list(self._pid) if self._have_event_id else None,
            event_time_zero=list(self._timestamps),
        )
        self.clear()
        return out

    def release_buffers(self) -> None:
        self._buffers_in_use = False

    def clear(self) -> None:
        self._toa.clear()
        self._pid.clear()
        self._timestamps.clear()


class StreamKind(str, Enum):
    """Subset of SRC/core/message.py StreamKind used on the hot path."""

    DETECTOR_EVENTS = 'detector_events'
    MONITOR_EVENTS = 'monitor_events'


@dataclass(frozen=True)
class StreamId:
    kind: StreamKind
    name: str


@dataclass
class GpuPreprocessorFactory:
    """``PreprocessorFactory.make_preprocessor`` for event streams.

    ``detector_numbers`` maps configured detector names to their
    ``detector_number`` arrays (``Instrument.get_detector_number``,
    SRC/config/instrument.py:415-416); unconfigured detectors are skipped by
    returning None, as the reference does (detector_data.py:44-47).
    """

    detector_numbers: dict[str, np.ndarray] = field(default_factory=dict)
    monitors: Sequence[str] = ()

    def make_preprocessor(self, key: StreamId) -> Any:
        if key.kind == StreamKind.DETECTOR_EVENTS:
            if key.name not in self.detector_numbers:
                return None
            return EventStaging(self.detector_numbers[key.name])
        if key.kind == StreamKind.MONITOR_EVENTS:
            return EventStaging()
        return None
