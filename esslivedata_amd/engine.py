"""Python handle of one HIP binning engine (thin wrapper over the C ABI).

One :class:`BinningEngine` holds the device state of one detector view or
monitor histogram: LUT, TOA thresholds, window and cumulative counts.  It is
single-thread-affine like the reference's jobs (SRC/core/job_manager.py:698-701).
"""

from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass

import numpy as np

from . import _native
from ._native import check
from .preprocessors import Timestamp


@dataclass
class FinalizeResult:
    current_image: np.ndarray | None
    cumulative_image: np.ndarray | None
    current_hist: np.ndarray | None
    cumulative_hist: np.ndarray | None
    current_total: int
    current_in_range: int
    cumulative_total: int
    cumulative_in_range: int


def _current_raw_stream(device_index: int) -> int:
    """hipStream_t of torch's current stream (cheap: no Stream object)."""
    import torch

    try:
        return int(torch._C._cuda_getCurrentRawStream(device_index))
    except AttributeError:  # pragma: no cover - older torch
        return int(torch.cuda.current_stream(device_index).cuda_stream)


class _HostBlock:
    """One ``lde_host_alloc`` block (page-locked, device-mapped host memory),
    exposed to numpy; freed when the last array viewing it is gone."""

    def __init__(self, nbytes: int, dtype: np.dtype, count: int) -> None:
        self._lib = _native.lib()
        p = ctypes.c_void_p()
        check(self._lib.lde_host_alloc(int(nbytes), ctypes.byref(p)), None, self._lib)
        self.ptr = int(p.value)
        self.__array_interface__ = {
            'shape': (count,), 'typestr': np.dtype(dtype).str, 'data': (self.ptr, False),
            'version': 3,
        }

    def __del__(self) -> None:
        try:
            self._lib.lde_host_free(self.ptr)
        except Exception:
            pass


class _OutputPool:
    """Finalize images the kernel writes in place (no host copy after the
    wait): arrays over ``lde_host_alloc`` blocks, handed out again only once
    nothing but the pool references them (a caller that keeps a result keeps
    its memory; a view of it counts as a reference).  At most ``cap`` blocks,
    beyond that finalize falls back to ordinary arrays and a copy.

    Ownership protocol: a caller keeps an image by keeping a Python reference
    to it (or to a numpy view of it).  A raw address alone (``a.ctypes.data``,
    ``__array_interface__`` consumers that keep no reference) does not keep
    the block, and the next finalize may overwrite it.  The reference count
    test is CPython's; on other interpreters, or with
    ``BinningEngine(reuse_output_buffers=False)``, every finalize returns fresh
    arrays (one host copy)."""

    def __init__(self, count: int, dtype: np.dtype, cap: int = 8, reuse: bool = True) -> None:
        import sys

        self._count, self._dtype, self._cap = count, np.dtype(dtype), cap
        self._arrays: list[np.ndarray] = []
        self._reuse = bool(reuse) and sys.implementation.name == 'cpython'

    def take(self) -> np.ndarray:
        import sys

        if not self._reuse:
            return np.empty(self._count, dtype=self._dtype)
        for a in self._arrays:
            # references: the pool's list, this loop variable, getrefcount's argument
            if sys.getrefcount(a) <= 3:
                return a
        if len(self._arrays) >= self._cap:
            return np.empty(self._count, dtype=self._dtype)
        a = np.asarray(_HostBlock(self._count * self._dtype.itemsize, self._dtype, self._count))
        self._arrays.append(a)
        return a


class PendingFinalize:
    """A finalize enqueued by ``BinningEngine.finalize(wait=False)``
    (``lde_finalize_begin``); ``result()`` waits for it alone
    (``lde_finalize_end``) and returns its :class:`FinalizeResult`."""

    def __init__(self, engine, ref, make) -> None:
        self._engine, self._ref, self._make, self._res = engine, ref, make, None

    def __del__(self) -> None:
        # dropped unread: complete it while its output arrays are still alive,
        # so the engine is not left with a pending finalize
        try:
            if self._res is None and getattr(self._engine, '_h', None) is not None:
                self.result()
        except Exception:
            pass

    def result(self) -> 'FinalizeResult':
        if self._res is None:
            e = self._engine
            if getattr(e, '_h', None) is None:
                raise RuntimeError('the engine was closed before this finalize was read')
            cur = getattr(e, '_pending', None)
            if cur is not None and cur() is self:
                e._pending = None
            rc = e._lib.lde_finalize_end(e._h, self._ref)
            if rc:
                check(rc, e._h, e._lib)
            self._res = self._make()
        return self._res


_I32_MIN, _I32_MAX = -(2**31), 2**31 - 1


def _as_i32(a, what: str, unknown_id: int | None = None) -> np.ndarray:
    """Contiguous int32 event array.  Wider integer arrays are converted
    only where their values fit: out-of-range pixel ids become
    ``unknown_id`` (an id outside the detector, so the event is dropped like
    any unknown id, group_by_pixel.py:46-54) instead of wrapping onto a valid
    pixel; out-of-range TOA values (the ev44 field is int32) are refused."""
    a = np.asarray(a)
    if a.dtype == np.int32:
        return np.ascontiguousarray(a)
    if a.dtype.kind not in 'iu':
        raise TypeError(f'event arrays must be integer, got {a.dtype}')
    if a.size == 0:
        return np.zeros(0, dtype=np.int32)
    if a.dtype.kind == 'u':
        bad = a > _I32_MAX
    else:
        bad = (a < _I32_MIN) | (a > _I32_MAX)
    if not bad.any():
        return np.ascontiguousarray(a, dtype=np.int32)
    if unknown_id is None:
        raise ValueError(f'{what} values must fit in int32')
    out = np.where(bad, 0, a).astype(np.int32)
    out[bad] = unknown_id
    return out


@dataclass
class DeviceMessages:
    """A batch's message descriptors (device pointers and lengths) and the
    tensors they point into (kept alive while staged)."""

    messages: list
    arr: object
    n: int


class BinningEngine:
    """Device-resident event binning for one view (see include/lde.h)."""

    def __init__(
        self,
        *,
        toa_edges_ns: np.ndarray,
        out_lut: np.ndarray | None,
        pid_offset: int = 0,
        n_screen: int = 1,
        out_dtype: str = 'float64',
        strategy: str = 'auto',
        toa_range: tuple[int, int] | None = None,
        device: int = 0,
        stream: int | None = None,  # hipStream_t; None/0: a torch pool stream
        reuse_output_buffers: bool = True,
    ) -> None:
        lib = _native.lib()
        edges = np.ascontiguousarray(np.asarray(toa_edges_ns, dtype=np.float64))
        if edges.ndim != 1 or len(edges) < 2:
            raise ValueError('toa edges need at least two values')
        self._T = len(edges) - 1
        self._S = int(n_screen)
        self._dtype = np.dtype(out_dtype)
        if self._dtype not in (np.dtype('float64'), np.dtype('float32')):
            raise ValueError('out_dtype must be float64 or float32')
        if strategy not in _native.STRATEGIES:
            raise ValueError(f'unknown strategy {strategy!r}')
        cfg = _native.LdeConfig()
        cfg.abi_version = _native.ABI_VERSION
        cfg.device_id = int(device)
        # The engine runs on a torch stream: the caller's (a raw hipStream_t
        # whose lifetime the caller guarantees) or, by default, a dedicated
        # stream from torch's per-device pool.  Pool streams are never
        # destroyed, so tensors staged from other streams can be recorded on
        # it for the caching allocator (record_stream) and outlive the engine;
        # an engine-created stream could not (lde_destroy destroys it).
        self._torch_stream = None
        if not stream:
            import torch

            self._torch_stream = torch.cuda.Stream(device=torch.device('cuda', int(device)))
            stream = self._torch_stream.cuda_stream
        cfg.stream = ctypes.c_void_p(stream)
        cfg.pid_offset = int(pid_offset)
        self._lut = None
        if out_lut is None:
            cfg.n_replicas = 1
            cfg.lut_len = 0
            cfg.out_lut = None
        else:
            lut = np.ascontiguousarray(np.asarray(out_lut, dtype=np.int32))
            if lut.ndim == 1:
                lut = lut[None, :]
            self._lut = lut
            cfg.n_replicas = lut.shape[0]
            cfg.lut_len = lut.shape[1]
            cfg.out_lut = lut.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        cfg.n_screen = self._S
        cfg.n_toa_bins = self._T
        cfg.toa_edges = edges.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        cfg.out_dtype = _native.LDE_F32 if self._dtype == np.float32 else _native.LDE_F64
        cfg.strategy = _native.STRATEGIES[strategy]
        if toa_range is None:
            cfg.range_lo, cfg.range_hi = -1, -1
        else:
            cfg.range_lo, cfg.range_hi = int(toa_range[0]), int(toa_range[1])
        self._n_replicas = cfg.n_replicas
        # a pixel id no LUT entry covers: stands in for ids beyond int32
        lo, hi = int(pid_offset), int(pid_offset) + int(cfg.lut_len)
        self._unknown_id = lo - 1 if lo > _I32_MIN else (hi if hi <= _I32_MAX else None)
        h = ctypes.c_void_p()
        rc = lib.lde_create(ctypes.byref(cfg), ctypes.byref(h))
        check(rc, None, lib)
        self._h = h
        self._lib = lib
        self._device = int(device)
        self._keepalive: list = []
        self._n_groups: dict[int, int] = {}
        self._img_pool = _OutputPool(self._S, self._dtype, reuse=reuse_output_buffers)
        self._out = _native.LdeOutputs()  # reused by finalize (every field set per call)
        self._out_ref = ctypes.byref(self._out)
        sp = ctypes.c_void_p()
        check(lib.lde_get_stream(h, ctypes.byref(sp)), h, lib)
        self._stream_ptr = int(sp.value or 0)

    # ------------------------------------------------------------------
    @classmethod
    def monitor(cls, toa_edges_ns: np.ndarray, **kwargs) -> 'BinningEngine':
        return cls(toa_edges_ns=toa_edges_ns, out_lut=None, n_screen=1, **kwargs)

    @property
    def n_screen(self) -> int:
        return self._S

    @property
    def n_toa_bins(self) -> int:
        return self._T

    @property
    def n_replicas(self) -> int:
        return self._n_replicas

    @property
    def dtype(self) -> np.dtype:
        return self._dtype

    def _call(self, fn, *args) -> None:
        check(fn(self._h, *args), self._h, self._lib)

    # ------------------------------------------------------------------
    def stage(self, pid, toa) -> None:
        """Stage one message of host events (ToNXevent_data.add equivalent)."""
        t = _as_i32(toa, 'time_of_arrival')
        if pid is None:
            self._call(self._lib.lde_stage, None, t.ctypes.data, len(t))
            return
        p = _as_i32(pid, 'pixel_id', self._unknown_id)
        if len(p) != len(t):
            raise ValueError(
                f'pixel_id and time_of_arrival must have the same length, '
                f'got {len(p)} and {len(t)}'
            )
        self._call(self._lib.lde_stage, p.ctypes.data, t.ctypes.data, len(t))

    def stage_ev44(self, payload, kafka_timestamp_ms: int = 0, *, single_pulse: bool = True):
        """Decode one ev44 payload in the engine and stage its events
        (``lde_stage_ev44``): the adapter chain plus ``ToNXevent_data.add`` in
        one native call.  Returns the message ``Timestamp``."""
        raw = np.frombuffer(payload, dtype=np.uint8) if not isinstance(payload, np.ndarray) else payload
        ts = ctypes.c_int64()
        flags = 1 if single_pulse else 0
        self._call(self._lib.lde_stage_ev44, raw.ctypes.data if raw.size else None, raw.size,
                   int(kafka_timestamp_ms), flags, ctypes.byref(ts))
        return Timestamp.from_ns(ts.value)

    def stage_device(self, pid_ptr: int | None, toa_ptr: int, n: int, keepalive=None) -> None:
        """Stage events already in HBM (device pointers, int32)."""
        if keepalive is not None:
            self._keepalive.append(keepalive)
        self._call(self._lib.lde_stage_device, pid_ptr, toa_ptr, int(n))

    @property
    def stream_ptr(self) -> int:
        """The hipStream_t (as an int) the engine's kernels run on."""
        return self._stream_ptr

    def _order_after_producer(self, tensors) -> None:
        """Device staging contract (include/lde.h, lde_stage_device): the
        engine stream waits for the producing (torch current) stream, and the
        caching allocator may not reuse the tensors' blocks before the engine
        stream has passed the kernels the next accumulate enqueues."""
        import torch

        dev = tensors[0].device
        cur = torch.cuda.current_stream(dev)
        if cur.cuda_stream == self._stream_ptr:
            return  # same stream: in order by construction
        if dev.index != self._device:
            raise ValueError(f'event tensors are on {dev}, the engine on device {self._device}')
        if self._torch_stream is None:
            self._torch_stream = torch.cuda.ExternalStream(self._stream_ptr, device=dev)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._torch_stream.wait_event(ev)
        for t in tensors:
            t.record_stream(self._torch_stream)

    def wait_event(self, event) -> None:
        """Make the engine stream wait for a ``torch.cuda.Event`` (no-op when
        the engine runs on torch's current stream, which is ordered anyway)."""
        import torch

        dev = torch.device('cuda', self._device)
        if _current_raw_stream(self._device) == self._stream_ptr:
            return
        if self._torch_stream is None:
            self._torch_stream = torch.cuda.ExternalStream(self._stream_ptr, device=dev)
        self._torch_stream.wait_event(event)

    @staticmethod
    def _check_event_tensor(t) -> None:
        import torch

        if t.dtype != torch.int32:
            raise ValueError(f'device event tensors must be contiguous int32, got {t.dtype}')
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError('device event tensors must be contiguous int32 on the GPU')

    def stage_tensors(self, pid, toa) -> None:
        """Stage int32 torch tensors resident on this engine's device."""
        if pid is not None and pid.numel() != toa.numel():
            raise ValueError('pixel_id and time_of_arrival must have the same length')
        ts = [t for t in (pid, toa) if t is not None]
        for t in ts:
            self._check_event_tensor(t)
        self._order_after_producer(ts)
        self.stage_device(
            None if pid is None else pid.data_ptr(), toa.data_ptr(), toa.numel(), (pid, toa)
        )

    def stage_tensors_batch(self, messages) -> None:
        """Stage a batch of ``(pid, toa)`` int32 device tensors in one call
        (``pid`` may be None for a monitor)."""
        if len(messages) == 0:
            return
        self.stage_device_messages(self.device_messages(messages))

    def device_messages(self, messages) -> 'DeviceMessages':
        """The descriptor table of a batch of ``(pid, toa)`` int32 device
        tensors (checked here), for :meth:`stage_device_messages`: a service
        builds it as the messages arrive, the engine stages it in one call."""
        import torch

        n = len(messages)
        # host time here is GPU idle time between batches: one pass over the
        # messages filling a ctypes array (pid pointers | toa pointers |
        # lengths), identity dtype test first (torch attribute calls dominate)
        i32 = torch.int32
        arr = (ctypes.c_int64 * (3 * n))()
        for i, (pid, toa) in enumerate(messages):
            if toa.dtype is not i32 or not toa.is_contiguous() or not toa.is_cuda:
                self._check_event_tensor(toa)
            nn = toa.numel()
            if pid is not None:
                if pid.dtype is not i32 or not pid.is_contiguous() or not pid.is_cuda:
                    self._check_event_tensor(pid)
                if pid.numel() != nn:
                    raise ValueError('pixel_id and time_of_arrival must have the same length')
                arr[i] = pid.data_ptr()
            arr[n + i] = toa.data_ptr()
            arr[2 * n + i] = nn
        return DeviceMessages(messages, arr, n)

    def stage_device_messages(self, table: 'DeviceMessages') -> None:
        """Stage a :meth:`device_messages` table (``lde_stage_device_batch``)."""
        n = table.n
        if n == 0:
            return
        msgs = table.messages
        if _current_raw_stream(msgs[0][1].device.index) != self._stream_ptr:
            self._order_after_producer([t for m in msgs for t in m if t is not None])
        base = ctypes.addressof(table.arr)
        rc = self._lib.lde_stage_device_batch(self._h, n, base, base + 8 * n, base + 16 * n)
        if rc:
            check(rc, self._h, self._lib)
        self._keepalive.append(msgs)

    def accumulate(self, replica: int = 0) -> None:
        rc = self._lib.lde_accumulate(self._h, int(replica))
        if rc:
            check(rc, self._h, self._lib)
        self._keepalive.clear()

    def finalize(self, *, images: bool = True, hists: bool = False, wait: bool = True):
        """Cumulative += window, the outputs, window cleared (``lde_finalize``).

        ``wait=False`` returns a :class:`PendingFinalize` at once: the finalize
        is enqueued and the window restarted, so the next ``accumulate`` can be
        enqueued before ``.result()`` waits for this window's outputs (the
        device bins the next batch while the host handles these).  One
        finalize may be pending per engine."""
        out = _native.LdeOutputs() if not wait else self._out
        ci = mi = ch = mh = None
        if images:
            # written in place by the finalize kernel (page-locked pool)
            ci = self._img_pool.take()
            mi = self._img_pool.take()
        if hists:
            ch = np.empty(self._S * self._T, dtype=self._dtype)
            mh = np.empty(self._S * self._T, dtype=self._dtype)
        out.current_image = ci.ctypes.data if ci is not None else None
        out.cumulative_image = mi.ctypes.data if mi is not None else None
        out.current_hist = ch.ctypes.data if ch is not None else None
        out.cumulative_hist = mh.ctypes.data if mh is not None else None
        ref = self._out_ref if wait else ctypes.byref(out)
        shape = (self._S, self._T)

        def result() -> FinalizeResult:
            t0, t1, t2, t3 = out.totals
            return FinalizeResult(
                current_image=ci,
                cumulative_image=mi,
                current_hist=ch.reshape(shape) if hists else None,
                cumulative_hist=mh.reshape(shape) if hists else None,
                current_total=t0,
                current_in_range=t1,
                cumulative_total=t2,
                cumulative_in_range=t3,
            )

        if wait:
            rc = self._lib.lde_finalize(self._h, ref)
            if rc:
                check(rc, self._h, self._lib)
            return result()
        rc = self._lib.lde_finalize_begin(self._h, ref)
        if rc:
            check(rc, self._h, self._lib)
        pending = PendingFinalize(self, ref, result)
        self._pending = weakref.ref(pending)  # (no cycle: the pending result holds the engine)
        return pending

    def read_histogram(self, which: str = 'current') -> np.ndarray:
        w = {'current': _native.LDE_CURRENT, 'cumulative': _native.LDE_CUMULATIVE}[which]
        out = np.empty(self._S * self._T, dtype=self._dtype)
        self._call(self._lib.lde_read_histogram, w, out.ctypes.data)
        return out.reshape(self._S, self._T)

    def clear(self) -> None:
        self._keepalive.clear()
        self._call(self._lib.lde_clear)

    def set_lut(self, out_lut: np.ndarray) -> None:
        """Replace the pid -> screen LUT (same shape as at construction)."""
        lut = np.ascontiguousarray(np.asarray(out_lut, dtype=np.int32))
        if lut.ndim == 1:
            lut = lut[None, :]
        if self._lut is None or lut.shape != self._lut.shape:
            raise ValueError(f'LUT shape {lut.shape} differs from the engine\'s '
                             f'{None if self._lut is None else self._lut.shape}')
        self._call(self._lib.lde_set_lut, lut.ctypes.data)
        self._lut = lut

    def set_coordinate_lut(self, pixel_distance, table, *, dist0: float, dist_step: float,
                           time0: float, time_step: float) -> None:
        """Wavelength mode (``lde_set_coord_lut``): events are histogrammed by
        the coordinate ``table`` (n_dist x n_time, bilinear) at their pixel's
        distance and their time of arrival (ns); the engine's edges are then
        in the coordinate's unit.  ``pixel_distance`` is per pixel id of the
        LUT (pid_offset + k), NaN where the pixel has no coordinate; a monitor
        engine takes one distance (its flight path) for all events."""
        d = np.ascontiguousarray(np.asarray(pixel_distance, dtype=np.float64))
        tab = np.ascontiguousarray(np.asarray(table, dtype=np.float64))
        if tab.ndim != 2:
            raise ValueError('table must be 2-D (distance, time)')
        lut = _native.LdeCoordLut()
        lut.pixel_distance = d.ctypes.data
        lut.n_pixels = d.size
        lut.table = tab.ctypes.data
        lut.n_dist, lut.n_time = tab.shape
        lut.dist0, lut.dist_step = float(dist0), float(dist_step)
        lut.time0, lut.time_step = float(time0), float(time_step)
        self._call(self._lib.lde_set_coord_lut, ctypes.byref(lut))

    def reset_cumulative(self) -> None:
        self._call(self._lib.lde_reset_cumulative)

    def finalize_partials(self, dst_ptr: int) -> None:
        """Finalize into device memory: uint64 [S] current image, [S]
        cumulative image, [4] totals (this rank's exact share, for a reduce)."""
        self._call(self._lib.lde_finalize_partials, dst_ptr)

    def accumulate_push(self, replica: int, dst_ptr: int) -> None:
        """Bin the staged events and write this push's exact counts (uint64
        [S*T]) to device memory instead of adding them (float32 views: the
        sharded per-push merge, ``lde_accumulate_push``)."""
        rc = self._lib.lde_accumulate_push(self._h, int(replica), dst_ptr)
        if rc:
            check(rc, self._h, self._lib)
        self._keepalive.clear()

    def push_counts(self, src_ptr: int) -> None:
        """Add one push of exact uint64 [S*T] counts to the float32 window and
        cumulative in the reference order (``lde_push_u64``)."""
        self._call(self._lib.lde_push_u64, src_ptr)

    def export_window(self, dst_ptr: int) -> None:
        self._call(self._lib.lde_export_window, dst_ptr)

    def import_window(self, src_ptr: int) -> None:
        self._call(self._lib.lde_import_window, src_ptr)

    def export_window_u64(self, dst_ptr: int) -> None:
        """Window counts as uint64 [S*T] into device memory (any window state)."""
        self._call(self._lib.lde_export_window_u64, dst_ptr)

    def import_window_u64(self, src_ptr: int) -> None:
        """Replace the window with uint64 [S*T] counts from device memory."""
        self._call(self._lib.lde_import_window_u64, src_ptr)

    def synchronize(self) -> None:
        self._call(self._lib.lde_synchronize)

    def set_groups(self, slot: int, groups) -> None:
        """Register screen groups (ROIs, spectrum-view output pixels) in ``slot``:
        ``groups`` is a sequence of flat screen-index arrays (may overlap)."""
        groups = [np.asarray(g, dtype=np.int32).ravel() for g in groups]
        offsets = np.zeros(len(groups) + 1, dtype=np.int64)
        if groups:
            offsets[1:] = np.cumsum([g.size for g in groups])
        screens = (np.concatenate(groups) if groups else np.zeros(0, np.int32)).astype(np.int32)
        screens = np.ascontiguousarray(screens)
        self._call(self._lib.lde_set_groups, int(slot), len(groups),
                   offsets.ctypes.data if groups else None,
                   screens.ctypes.data if screens.size else None)
        self._n_groups[int(slot)] = len(groups)

    def group_spectra(self, slot: int, which: str = 'current') -> np.ndarray:
        """``(n_groups, T)`` spectra of the groups in ``slot`` from the window
        (``'current'``) or the cumulative including the window."""
        w = {'current': _native.LDE_CURRENT, 'cumulative': _native.LDE_CUMULATIVE}[which]
        n = self._n_groups.get(int(slot), 0)
        out = np.zeros((n, self._T), dtype=self._dtype)
        self._call(self._lib.lde_group_spectra, int(slot), w, out.ctypes.data if n else None)
        return out

    def timing_select(self, kernels=None) -> None:
        """Record only these kernel ids (names of _native.KERNELS); None = all."""
        mask = 0xFFFFFFFF if kernels is None else sum(1 << _native.KERNELS[k] for k in kernels)
        self._call(self._lib.lde_timing_select, mask)

    def timing_enable(self, enable: bool = True) -> None:
        self._call(self._lib.lde_timing_enable, 1 if enable else 0)

    def kernel_stats(self, kernel: str) -> tuple[float, int]:
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        self._call(
            self._lib.lde_kernel_stats, _native.KERNELS[kernel], ctypes.byref(ms), ctypes.byref(n)
        )
        return ms.value, n.value

    def counter(self, name: str) -> int:
        """An engine counter (``lde_counter``; names in ``_native.COUNTERS``)."""
        v = ctypes.c_int64()
        self._call(self._lib.lde_counter, _native.COUNTERS[name], ctypes.byref(v))
        return v.value

    def info(self) -> dict:
        s, st, eb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        t, tb, nt, ls = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._call(
            self._lib.lde_info,
            ctypes.byref(s),
            ctypes.byref(t),
            ctypes.byref(st),
            ctypes.byref(tb),
            ctypes.byref(nt),
            ctypes.byref(eb),
            ctypes.byref(ls),
        )
        return {
            'n_screen': s.value,
            'n_toa_bins': t.value,
            'staged': st.value,
            'tile_bits': tb.value,
            'n_tiles': nt.value,
            'events_binned': eb.value,
            'last_strategy': {0: 'monitor', 1: 'atomic', 2: 'partition', 3: 'paged', 4: 'split', 5: 'pixel', 6: 'wide'}.get(ls.value, '?'),
            'device': self._device,
        }

    def close(self) -> None:
        h = getattr(self, '_h', None)
        if h:
            ref = getattr(self, '_pending', None)
            p = ref() if ref is not None else None
            if p is not None:  # its outputs first (the pack dies with the handle)
                try:
                    p.result()
                except Exception:
                    pass
            self._lib.lde_destroy(h)
            self._h = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass
