"""Workflow-protocol side of the drop-in boundary (GPU detector view / monitor).

``GpuDetectorViewWorkflow`` and ``GpuMonitorWorkflow`` implement the
reference's ``Workflow`` protocol (SRC/workflows/workflow_factory.py:22-34:
``accumulate(data, *, start_time, end_time)``, ``finalize() -> dict``,
``clear()``) plus ``SupportsContext.build`` (:37-57), with the same output
names (SRC/workflows/detector_view/factory.py:208-215,
SRC/workflows/monitor_workflow.py:318-325) and window time coords
(SRC/workflows/stream_processor_workflow.py:225-244).  Every per-event step
runs in the HIP engine (``BinningEngine``); the host only stages message
arrays and assembles the small finalize outputs.

Semantics mirrored:
* replica cycling ``counter % R`` per accumulate (projectors.py:105-113);
* cumulative/current pair with reset-on-geometry-change
  (SRC/preprocessors/accumulators.py:86-195);
* ``detector_image``: sum over the TOA slice, optional ``/ weights``;
  ``counts_total``; ``counts_in_range`` (providers.py:236-357);
* monitor histogram coord: edges converted to ns and back to the edge unit
  (monitor_workflow.py:93-100), ranges by label slicing (:154-167).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import TYPE_CHECKING, Any, Callable, Iterable, Mapping, Sequence

import numpy as np

from .dataarray import DataArray, Variable, publish
from .edges import TOAEdges, WavelengthEdges, convert_time, convert_wavelength, label_slice
from .engine import BinningEngine
from .preprocessors import DetectorEvents, MonitorEvents, StagedEvents, Timestamp
from .projection import ViewLUT, geometric_lut, index_groups, logical_lut

if TYPE_CHECKING:
    from .geometry import GeometricSource
    from .wavelength import WavelengthLookupTable
from . import roi as _roi

DETECTOR_TRANSFORM = 'detector_transform'
MONITOR_TRANSFORM = 'monitor_transform'

DETECTOR_WINDOW_OUTPUTS = ('current', 'counts_total', 'counts_in_toa_range')
# with ROI support the current ROI spectra are window outputs too
# (DetectorViewOutputs.fields_with(Temporality.window), detector_view/factory.py:262-276)
ROI_WINDOW_OUTPUTS = ('roi_spectra_current',)
TOA_DIM = 'time_of_arrival'
WAVELENGTH_DIM = 'wavelength'
_ROI_SLOT = 0
_SPECTRUM_SLOT = 1
MONITOR_WINDOW_OUTPUTS = ('current', 'counts_total', 'counts_in_toa_range')


# ---------------------------------------------------------------------------
# parameters and view configuration
# ---------------------------------------------------------------------------
@dataclass
class DetectorViewParams:
    """``DetectorViewParams`` (SRC/workflows/detector_view_specs.py:53-124):
    ``coordinate_mode`` 'toa' or 'wavelength' selects which edges and range
    are active (``get_active_edges`` / ``get_active_range``, :106-124)."""

    toa_edges: TOAEdges = field(default_factory=TOAEdges)
    toa_range: tuple[float, float] | None = None  # in toa_edges.unit; None = disabled
    pixel_weighting: bool = False
    coordinate_mode: str = 'toa'
    wavelength_edges: WavelengthEdges = field(default_factory=WavelengthEdges)
    wavelength_range: tuple[float, float] | None = None  # in wavelength_edges.unit

    def __post_init__(self) -> None:
        if self.coordinate_mode not in ('toa', 'wavelength'):
            raise ValueError(f"coordinate_mode must be 'toa' or 'wavelength', "
                             f"got {self.coordinate_mode!r}")

    def get_active_edges(self) -> TOAEdges | WavelengthEdges:
        return self.wavelength_edges if self.coordinate_mode == 'wavelength' else self.toa_edges

    def get_active_range(self) -> tuple[float, float] | None:
        return self.wavelength_range if self.coordinate_mode == 'wavelength' else self.toa_range


@dataclass(frozen=True)
class GeometricViewConfig:
    """``GeometricViewConfig`` (SRC/workflows/detector_view/types.py:94-131)."""

    projection_type: str
    resolution: dict[str, int]
    pixel_noise: Any = None
    flip_x: bool = False


@dataclass(frozen=True)
class LogicalViewConfig:
    """``LogicalViewConfig`` (SRC/workflows/detector_view/types.py:100-126).

    ``transform(da, source_name)`` receives a :class:`logical.LogicalIndex`
    (the pixel indices with the detector's dims) and folds / transposes /
    slices / flattens it with the scipp calls the reference's transforms use;
    ``reduction_dim`` (a dim name or a list of names) is merged as
    ``bins.concat`` does (projectors.py:243-270).  A transform that returns a
    plain array instead names its merged axes by position in
    ``reduction_axes``."""

    transform: Callable[[Any, str], Any] | None = None
    reduction_dim: str | Sequence[str] | None = None
    reduction_axes: Sequence[int] = ()
    output_dims: tuple[str, ...] | None = None
    roi_support: bool = True
    spectrum_view: 'SpectrumViewConfig | None' = None


@dataclass(frozen=True)
class SpectrumViewConfig:
    """``SpectrumViewSpec`` (SRC/workflows/detector_view/types.py) in index form.

    The reference's transform folds / sums / flattens the cumulative
    ``(screen..., toa)`` histogram (providers.py:300-325; BIFROST
    bifrost/specs.py:311-329).  Here ``transform`` receives the flat screen
    index array of shape ``screen_shape`` and returns it folded / transposed;
    ``reduction_axes`` of the result are summed; ``output_dims`` name the kept
    axes.  The regrouping then runs on the GPU (``lde_group_spectra``).
    """

    transform: Callable[[np.ndarray], np.ndarray] | None
    output_dims: tuple[str, ...]
    reduction_axes: Sequence[int] = ()


def _stamp_window(out: dict, names: Sequence[str], start: Timestamp | None,
                  end: Timestamp | None) -> None:
    """Window outputs get 0-D ``start_time`` (first accumulate since the last
    finalize) and ``time`` (last end) coords: int64 scalars with unit 'ns', as
    ``Timestamp.to_scipp()`` makes them (SRC/workflows/stream_processor_workflow.py:
    229-238, SRC/core/timestamp.py:216-220); cumulative outputs stay unstamped
    (``Job._add_time_coords`` stamps them, SRC/core/job.py:212-262)."""
    if start is None:
        return
    st, tt = start.to_scipp(), end.to_scipp()
    for name in names:
        if name in out:
            out[name] = out[name].assign_coords(start_time=st, time=tt)


def _histogram_slice(edges, toa_range) -> tuple[int, int] | None:
    if toa_range is None:
        return None
    return label_slice(edges.get_edges(), float(toa_range[0]), float(toa_range[1]))


def _events_of(data) -> tuple[list, list | None]:
    """Normalise the accepted inputs into per-message (pid, toa) lists."""
    if isinstance(data, StagedEvents):
        return data.time_of_arrival, data.pixel_id
    if isinstance(data, DetectorEvents):
        return [data.time_of_arrival], [data.pixel_id]
    if isinstance(data, MonitorEvents):
        return [data.time_of_arrival], None
    if isinstance(data, tuple) and len(data) == 2:
        pid, toa = data
        return [toa], None if pid is None else [pid]
    raise TypeError(f'unsupported event payload {type(data).__name__}')


def _stage(engine: BinningEngine, toas: list, pids: list | None) -> None:
    if toas and all(hasattr(t, 'data_ptr') for t in toas):  # device tensors: one call, no copy
        engine.stage_tensors_batch([(None if pids is None else pids[i], t) for i, t in enumerate(toas)])
        return
    for i, toa in enumerate(toas):
        pid = None if pids is None else pids[i]
        if hasattr(toa, 'data_ptr'):  # device tensors: no copy
            engine.stage_tensors(pid, toa)
        else:
            engine.stage(pid, toa)


class _ContextState:
    """Tracks the geometry signal context (reset-on-move)."""

    def __init__(self, key: str | None) -> None:
        self.key = key
        self.value = None

    def changed(self, data: Mapping[str, Any]) -> bool:
        if self.key is None or self.key not in data:
            return False
        new = data[self.key]
        old, self.value = self.value, new
        if old is None or new is None:
            return False
        return not np.array_equal(np.asarray(old), np.asarray(new))


# ---------------------------------------------------------------------------
# detector view
# ---------------------------------------------------------------------------
class GpuDetectorViewWorkflow:
    """Detector view (TOA or wavelength mode) on the MI355X engine."""

    def __init__(
        self,
        source_name: str,
        view: ViewLUT,
        params: DetectorViewParams | None = None,
        *,
        out_dtype: str = 'float64',
        device: int = 0,
        stream: int | None = None,
        geometry_key: str | None = DETECTOR_TRANSFORM,
        strategy: str = 'auto',
        roi_support: bool = False,
        roi_keys: Mapping[str, str] | None = None,
        spectrum_view: SpectrumViewConfig | None = None,
        geometry: 'GeometricSource | None' = None,
        lookup_table: 'WavelengthLookupTable | None' = None,
        source_position=(0.0, 0.0, -76.55),
        sample_position=(0.0, 0.0, 0.0),
    ) -> None:
        self._source = source_name
        # geometric views built from positions rebuild their LUT when the
        # detector transform (the geometry signal) changes
        self._geometry_src = geometry
        if view is None:
            if geometry is None:
                raise ValueError('a view LUT or a geometry is required')
            view = geometry.view()
        self._view = view
        self._params = params or DetectorViewParams()
        edges = self._params.get_active_edges()
        self._wavelength = self._params.coordinate_mode == 'wavelength'
        if self._wavelength:
            # factory.py:134-142: wavelength mode needs the lookup table and
            # the geometry (Ltotal per pixel)
            if lookup_table is None:
                raise ValueError('wavelength mode requires a lookup table')
            if geometry is None:
                raise ValueError('wavelength mode requires geometry for Ltotal computation')
            engine_edges = edges.edges_in(lookup_table.unit)
            self._spec_dim = WAVELENGTH_DIM
        else:
            engine_edges = edges.edges_ns()
            self._spec_dim = TOA_DIM
        self._lookup = lookup_table
        self._beamline = (source_position, sample_position)
        self._spec_edges = edges
        self._edges_unit = edges.get_edges()
        self._slice = _histogram_slice(edges, self._params.get_active_range())
        self._engine = BinningEngine(
            toa_edges_ns=engine_edges,
            out_lut=view.lut,
            pid_offset=view.pid_offset,
            n_screen=view.n_screen,
            out_dtype=out_dtype,
            strategy=strategy,
            toa_range=self._slice,
            device=device,
            stream=stream,
        )
        if self._wavelength:
            self._set_coordinates()
        self._counter = 0
        self._geometry = _ContextState(geometry_key)
        self._context_keys: dict[str, Any] = {}
        self._built = False
        self._start: Timestamp | None = None
        self._end: Timestamp | None = None
        # ROI requests arrive as context streams keyed by their wire names
        # (aux_source_names, detector_view/factory.py:234-246)
        self._roi_support = roi_support
        keys = dict(roi_keys or {})
        self._roi_keys = {'roi_rectangle': keys.get('roi_rectangle', 'roi_rectangle'),
                          'roi_polygon': keys.get('roi_polygon', 'roi_polygon')}
        self._roi_requests: dict[str, Any] = {'roi_rectangle': None, 'roi_polygon': None}
        self._roi_index: list[int] = []
        self._spectrum = spectrum_view
        self._spectrum_shape: tuple[int, ...] = ()
        if spectrum_view is not None:
            shape, groups = index_groups(view.screen_shape, spectrum_view.transform,
                                         spectrum_view.reduction_axes)
            if len(shape) != len(spectrum_view.output_dims):
                raise ValueError(f'spectrum view output_dims {spectrum_view.output_dims} do not '
                                 f'match the transformed shape {shape}')
            self._spectrum_shape = shape
            self._engine.set_groups(_SPECTRUM_SLOT, groups)

    @property
    def engine(self) -> BinningEngine:
        return self._engine

    @property
    def view(self) -> ViewLUT:
        return self._view

    # SupportsContext
    def build(self, *, context_keys: Mapping[str, Any] | None = None,
              chain_patch_bindings: Iterable = ()) -> None:
        bindings = list(chain_patch_bindings)
        if self._built:
            if context_keys or bindings:
                raise RuntimeError('Cannot inject bindings: the workflow is already built.')
            return
        if context_keys:
            self._context_keys.update(context_keys)
        self._built = True

    def accumulate(self, data: dict[str, Any], *, start_time: Timestamp,
                   end_time: Timestamp) -> None:
        self._accumulate(data, start_time, end_time)

    def _accumulate(self, data: Mapping[str, Any], start_time: Timestamp, end_time: Timestamp,
                    batch_has_events: bool = False, bin_fn=None) -> None:
        """``batch_has_events``: another rank binned events of this batch (the
        sharded workflow), so the replica cycle advances here too.
        ``bin_fn(replica)`` bins the staged events instead of
        ``engine.accumulate`` (the sharded per-push merge)."""
        if self._start is None:
            self._start = start_time
        self._end = end_time
        if self._geometry_src is not None and self._geometry.key in data:
            self._move(data[self._geometry.key])
        if self._geometry.changed(data):
            self._engine.reset_cumulative()
        if self._roi_support:
            self._update_rois(data)
        if self._source not in data:
            if batch_has_events:
                self._counter += 1  # one replica per batch (projectors.py:105-113)
            return
        toas, pids = _events_of(data[self._source])
        if pids is None:
            raise ValueError('detector events need pixel ids')
        _stage(self._engine, toas, pids)
        replica = self._counter % self._view.n_replicas
        self._counter += 1
        (bin_fn or self._engine.accumulate)(replica)

    def _move(self, transform) -> None:
        """A detector-transform value: rebuild the projection and LUT from the
        moved positions when it differs from the current placement (the
        reference rebuilds its projector from the re-resolved positions)."""
        geo = self._geometry_src
        t = None if transform is None else np.asarray(getattr(transform, 'values', transform))
        cur = geo.transform
        if t is None or (cur is not None and np.array_equal(np.asarray(cur), t)):
            return
        # build and validate the moved view before anything is committed, so a
        # rejected move leaves geometry, LUT and coordinates at the old placement
        view = geo.view(t)
        if view.screen_shape != self._view.screen_shape or view.n_replicas != self._view.n_replicas:
            raise ValueError('a detector move cannot change the view shape')
        self._engine.set_lut(view.lut)
        geo.transform = t
        self._view = view
        if self._wavelength:
            self._set_coordinates()  # Ltotal moved with the detector
        if self._roi_support and any(r is not None for r in self._roi_requests.values()):
            # the ROI masks are screen metadata of the moved projection
            # (precompute_roi_rectangle_bounds / _polygon_masks, roi.py:31-125)
            self._set_roi_groups()

    def _set_coordinates(self) -> None:
        """Per-pixel Ltotal of the current placement + the table -> engine."""
        from .wavelength import distance_per_pid, pixel_ltotal

        geo, tab = self._geometry_src, self._lookup
        src, smp = self._beamline
        lt = pixel_ltotal(geo.pixel_positions(), source_position=src, sample_position=smp)
        d = distance_per_pid(geo.detector_number, lt, self._view.pid_offset,
                             self._view.lut.shape[1])
        self._engine.set_coordinate_lut(d, tab.table, dist0=tab.distance0,
                                        dist_step=tab.distance_step, time0=tab.time0,
                                        time_step=tab.time_step)

    def _update_rois(self, data: Mapping[str, Any]) -> None:
        """New ROI requests -> screen groups on the device (the reference's
        precompute_roi_rectangle_bounds / precompute_roi_polygon_masks, roi.py:31-125)."""
        changed = False
        for name, wire in self._roi_keys.items():
            if wire in data:
                self._roi_requests[name] = data[wire]
                changed = True
        if changed:
            self._set_roi_groups()

    def _set_roi_groups(self) -> None:
        rects = _roi.from_concatenated(self._roi_requests['roi_rectangle'])
        polys = _roi.from_concatenated(self._roi_requests['roi_polygon'])
        self._roi_index, groups = _roi.roi_groups(self._view, rects, polys)
        self._engine.set_groups(_ROI_SLOT, groups)

    def _toa_coord(self) -> Variable:
        """The spectral coord: TOA or wavelength edges in the edges' unit."""
        return Variable((self._spec_dim,), self._edges_unit, self._spec_edges.unit)

    def _roi_spectra(self, which: str) -> DataArray:
        """``roi_spectra`` (roi.py:188-266): dims (roi, toa), int32 roi coord."""
        n = len(self._roi_index)
        if n:
            values = self._engine.group_spectra(_ROI_SLOT, which)
        else:
            values = np.zeros((0, self._engine.n_toa_bins), dtype=self._engine.dtype)
        return DataArray(values, ('roi', self._spec_dim), 'counts', {
            'roi': Variable(('roi',), np.asarray(self._roi_index, dtype=np.int32)),
            self._spec_dim: self._toa_coord(),
        })

    def _roi_readback(self, name: str) -> DataArray:
        """``roi_rectangle_readback`` / ``roi_polygon_readback`` (roi.py:293-353):
        the request unchanged, or an empty one carrying the screen coord units."""
        req = self._roi_requests[name]
        kind = 'rectangle' if name == 'roi_rectangle' else 'polygon'
        if isinstance(req, DataArray) and len(np.atleast_1d(req.values)) > 0:
            return req
        if isinstance(req, Mapping) and req:
            return _roi.to_concatenated(req, kind)
        y_dim, x_dim = (self._view.screen_dims + (None, None))[:2]
        units = {'x': self._view.screen_units.get(x_dim), 'y': self._view.screen_units.get(y_dim)}
        return _roi.to_concatenated({}, kind, coord_units=units)

    def _image(self, values: np.ndarray) -> DataArray:
        img = values.reshape(self._view.screen_shape)
        if self._params.pixel_weighting and self._view.pixel_weights is not None:
            with np.errstate(divide='ignore', invalid='ignore'):
                img = img / self._view.pixel_weights
        units = self._view.screen_units
        coords = {d: Variable((d,), c, units.get(d)) for d, c in self._view.screen_coords.items()}
        return DataArray(img, self._view.screen_dims, 'counts', coords)

    def finalize(self) -> dict[str, Any]:
        # grouped spectra read the window before finalize clears it; with an
        # empty window they raise the same ValueError finalize would
        extra: dict[str, Any] = {}
        if self._roi_support:
            extra['roi_spectra_current'] = self._roi_spectra('current')
            extra['roi_spectra_cumulative'] = self._roi_spectra('cumulative')
        if self._spectrum is not None:
            vals = self._engine.group_spectra(_SPECTRUM_SLOT, 'cumulative')
            extra['spectrum_view'] = DataArray(
                vals.reshape(*self._spectrum_shape, -1),
                (*self._spectrum.output_dims, self._spec_dim), 'counts',
                {self._spec_dim: self._toa_coord()},
            )
        res = self._engine.finalize(images=True)
        totals = (res.current_total, res.current_in_range, res.cumulative_total,
                  res.cumulative_in_range)
        return self._outputs(res.current_image, res.cumulative_image, totals, extra)

    def _outputs(self, current_image, cumulative_image, totals, extra=None) -> dict[str, Any]:
        """The published outputs from the window's and the cumulative's images
        and the four totals (current, current in range, cumulative,
        cumulative in range); also used by the sharded workflow on the merged
        partial outputs."""
        dt = self._engine.dtype.type
        cur_t, cur_r, cum_t, cum_r = totals
        out = {
            'cumulative': self._image(cumulative_image),
            'current': self._image(current_image),
            'counts_total': DataArray(np.asarray(dt(cur_t)), (), 'counts'),
            'counts_in_toa_range': DataArray(np.asarray(dt(cur_r)), (), 'counts'),
            'counts_total_cumulative': DataArray(np.asarray(dt(cum_t)), (), 'counts'),
            'counts_in_toa_range_cumulative': DataArray(np.asarray(dt(cum_r)), (), 'counts'),
        }
        out.update(extra or {})
        if self._roi_support:
            out['roi_rectangle'] = self._roi_readback('roi_rectangle')
            out['roi_polygon'] = self._roi_readback('roi_polygon')
        names = DETECTOR_WINDOW_OUTPUTS + (ROI_WINDOW_OUTPUTS if self._roi_support else ())
        _stamp_window(out, names, self._start, self._end)
        self._start = self._end = None
        return publish(out)

    @property
    def source_name(self) -> str:
        return self._source

    @property
    def has_grouped_outputs(self) -> bool:
        """ROI spectra or a spectrum view (read from the full histograms)."""
        return self._roi_support or self._spectrum is not None

    def _end_window(self) -> None:
        """Window bookkeeping of a finalize whose outputs are produced elsewhere."""
        self._start = self._end = None

    def read_histogram(self, which: str = 'cumulative') -> DataArray:
        h = self._engine.read_histogram(which)
        dims = (*self._view.screen_dims, self._spec_dim)
        shape = (*self._view.screen_shape, h.shape[-1])
        return DataArray(h.reshape(shape), dims, 'counts', {self._spec_dim: self._toa_coord()})

    def clear(self) -> None:
        self._engine.clear()
        self._start = self._end = None


class GpuDetectorViewFactory:
    """``DetectorViewFactory.make_workflow`` (detector_view/factory.py:95-276).

    ``detector_numbers`` supplies each source's ``detector_number`` (as
    ``Instrument.get_detector_number`` does); geometric views additionally
    need per-replica projected coordinates ``projected_coords[source][dim]`` of
    shape (replica, pixel), the output of essreduce's projection of
    ``CalibratedPositionWithNoisyReplicas`` (setup-time input).
    """

    def __init__(
        self,
        *,
        detector_numbers: Mapping[str, np.ndarray],
        view_config: GeometricViewConfig | LogicalViewConfig | Mapping[str, Any],
        projected_coords: Mapping[str, Mapping[str, np.ndarray]] | None = None,
        positions: Mapping[str, np.ndarray] | None = None,
        pixel_shapes: Mapping[str, Mapping[str, Any]] | None = None,
        transforms: Mapping[str, Any] | None = None,
        lookup_table: 'WavelengthLookupTable | None' = None,
        source_position=(0.0, 0.0, -76.55),
        sample_position=(0.0, 0.0, 0.0),
        out_dtype: str = 'float64',
        device: int = 0,
        detector_dims: Mapping[str, Sequence[str]] | None = None,
        strategy: str = 'auto',
    ) -> None:
        self._dn = dict(detector_numbers)
        self._strategy = strategy
        # wavelength mode: the (Ltotal, time) table (the reference's
        # LookupTableFilename) and the beamline for Ltotal
        self._lookup = lookup_table
        self._beamline = (source_position, sample_position)
        self._cfg = view_config
        self._coords = dict(projected_coords or {})
        # calibrated pixel positions (offsets in the component frame when a
        # transform is given) -> projection + noise replicas (geometry.py)
        self._positions = dict(positions or {})
        self._pixel_shapes = dict(pixel_shapes or {})
        self._transforms = dict(transforms or {})
        self._dtype = out_dtype
        self._device = device
        # dim names of each detector_number (1-D: 'detector_number')
        self._dims = dict(detector_dims or {})

    def make_geometry(self, source_name: str) -> 'GeometricSource':
        from .geometry import GeometricSource

        cfg = self._config(source_name)
        return GeometricSource(
            np.asarray(self._dn[source_name]), self._positions[source_name],
            projection_type=cfg.projection_type, resolution=cfg.resolution,
            pixel_noise=cfg.pixel_noise, flip_x=cfg.flip_x,
            pixel_shape=self._pixel_shapes.get(source_name),
            transform=self._transforms.get(source_name))

    def _config(self, source: str):
        if isinstance(self._cfg, Mapping):
            return self._cfg[source]
        return self._cfg

    def make_view(self, source_name: str) -> ViewLUT:
        cfg = self._config(source_name)
        dn = np.asarray(self._dn[source_name])
        if isinstance(cfg, GeometricViewConfig):
            if source_name in self._positions:
                return self.make_geometry(source_name).view()
            if source_name not in self._coords:
                raise ValueError(f'no positions or projected coordinates for {source_name!r}')
            return geometric_lut(dn, self._coords[source_name], cfg.resolution, flip_x=cfg.flip_x)
        if isinstance(cfg, LogicalViewConfig):
            tf = None if cfg.transform is None else (lambda a: cfg.transform(a, source_name))
            return logical_lut(dn, transform=tf, reduction_axes=cfg.reduction_axes,
                               reduction_dim=cfg.reduction_dim, output_dims=cfg.output_dims,
                               dims=self._dims.get(source_name))
        raise TypeError(f'unknown view config {type(cfg).__name__}')

    def make_workflow(self, source_name: str, params: DetectorViewParams | None = None,
                      aux_source_names: Mapping[str, str] | None = None) -> GpuDetectorViewWorkflow:
        cfg = self._config(source_name)
        # geometric views always support ROIs (factory.py:187); logical views per config
        roi_support = isinstance(cfg, GeometricViewConfig) or bool(cfg.roi_support)
        spectrum = cfg.spectrum_view if isinstance(cfg, LogicalViewConfig) else None
        geometry = None
        if isinstance(cfg, GeometricViewConfig) and source_name in self._positions:
            geometry = self.make_geometry(source_name)
        return GpuDetectorViewWorkflow(
            source_name, None if geometry is not None else self.make_view(source_name), params,
            out_dtype=self._dtype, device=self._device, strategy=self._strategy,
            roi_support=roi_support,
            roi_keys=aux_source_names, spectrum_view=spectrum, geometry=geometry,
            lookup_table=self._lookup, source_position=self._beamline[0],
            sample_position=self._beamline[1],
        )


# ---------------------------------------------------------------------------
# monitor histogram
# ---------------------------------------------------------------------------
class GpuMonitorWorkflow:
    """Monitor histogram (``create_monitor_workflow``, monitor_workflow.py:
    225-331): TOA mode, or wavelength mode (``histogram_wavelength_monitor``,
    :126-132) with the monitor's one flight path ``monitor_distance`` (m)
    through the lookup table."""

    def __init__(
        self,
        source_name: str,
        edges: TOAEdges | WavelengthEdges,
        *,
        range_filter: tuple[float, float] | None = None,
        coordinate_mode: str = 'toa',
        lookup_table: 'WavelengthLookupTable | None' = None,
        monitor_distance: float | None = None,
        device: int = 0,
        stream: int | None = None,
        geometry_key: str | None = MONITOR_TRANSFORM,
    ) -> None:
        self._source = source_name
        self._edges = edges
        if coordinate_mode not in ('toa', 'wavelength'):
            raise ValueError(f'Unsupported coordinate mode: {coordinate_mode}')
        self._wavelength = coordinate_mode == 'wavelength'
        e_unit = edges.get_edges()
        if self._wavelength:
            if lookup_table is None or monitor_distance is None:
                raise ValueError('wavelength mode requires a lookup table and the monitor distance')
            if not isinstance(edges, WavelengthEdges):
                raise ValueError('wavelength mode needs WavelengthEdges')
            e_ev = edges.edges_in(lookup_table.unit)
            # output coord: the edges in the event unit, converted back
            # (monitor_workflow.py:98-100)
            self._coord = convert_wavelength(e_ev, lookup_table.unit, edges.unit)
            self._dim = 'wavelength'
        else:
            e_ev = edges.edges_ns()
            # output coord: edges converted to ns and back (monitor_workflow.py:100)
            self._coord = convert_time(e_ev, 'ns', edges.unit)
            self._dim = 'time_of_arrival'
        lo, hi = range_filter if range_filter is not None else (e_unit[0], e_unit[-1])
        self._slice = label_slice(self._coord, float(lo), float(hi))
        self._engine = BinningEngine.monitor(e_ev, toa_range=self._slice, device=device,
                                             stream=stream)
        if self._wavelength:
            t = lookup_table
            self._engine.set_coordinate_lut([float(monitor_distance)], t.table, dist0=t.distance0,
                                            dist_step=t.distance_step, time0=t.time0,
                                            time_step=t.time_step)
        self._geometry = _ContextState(geometry_key)
        self._start: Timestamp | None = None
        self._end: Timestamp | None = None
        self._built = False
        self._device = device
        # histogram mode (da00 monitor histograms): float64 window and
        # cumulative on the device, fed by lde_rebin_f64
        self._hist_mode = False
        self._hcur = self._hcum = self._hedges = None
        self._hslice = label_slice(e_unit, float(lo), float(hi))
        self._hdata = False

    @property
    def engine(self) -> BinningEngine:
        return self._engine

    def _push_histogram(self, hist: DataArray) -> None:
        """Histogram mode (monitor_workflow.py:101-108): convert the coord to
        the edges' unit, rebin onto the edges and push into both accumulators
        on the GPU (one ``lde_rebin_f64`` launch)."""
        import torch

        from ._native import check, lib

        if self._wavelength:
            raise NotImplementedError('histogram-mode monitors are rebinned in TOA mode only')
        dim = hist.dims[0]
        coord = hist.coords[dim]
        src_edges = convert_time(np.asarray(coord.values, dtype=np.float64), coord.unit,
                                 self._edges.unit)
        vals = np.ascontiguousarray(hist.values, dtype=np.float64).reshape(-1)
        if src_edges.shape != (vals.size + 1,):
            raise ValueError(f'histogram coord {dim!r} must hold bin edges')
        dev = torch.device('cuda', self._device)
        if self._hcur is None:
            e = self._edges.get_edges()
            self._hedges = torch.as_tensor(np.asarray(e, dtype=np.float64), device=dev)
            self._hcur = torch.zeros(len(e) - 1, dtype=torch.float64, device=dev)
            self._hcum = torch.zeros_like(self._hcur)
        se = torch.as_tensor(src_edges, device=dev)
        sv = torch.as_tensor(vals, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        check(lib().lde_rebin_f64(se.data_ptr(), sv.data_ptr(), vals.size, self._hedges.data_ptr(),
                                  self._hcur.numel(), self._hcur.data_ptr(), self._hcum.data_ptr(),
                                  stream))
        torch.cuda.current_stream(dev).synchronize()  # se/sv are freed on return
        self._hist_mode = True
        self._hdata = True

    def build(self, *, context_keys=None, chain_patch_bindings: Iterable = ()) -> None:
        if self._built and (context_keys or list(chain_patch_bindings)):
            raise RuntimeError('Cannot inject bindings: the workflow is already built.')
        self._built = True

    def accumulate(self, data: dict[str, Any], *, start_time: Timestamp,
                   end_time: Timestamp) -> None:
        if self._start is None:
            self._start = start_time
        self._end = end_time
        if self._geometry.changed(data):
            self._engine.reset_cumulative()
            if self._hcum is not None:
                self._hcum.zero_()
                self._hcur.zero_()
        if self._source not in data:
            return
        value = data[self._source]
        if isinstance(value, DataArray) and np.ndim(value.values) == 1 and value.dims \
                and value.dims[0] in value.coords:
            self._push_histogram(value)
            return
        toas, _ = _events_of(value)
        _stage(self._engine, toas, None)
        self._engine.accumulate(0)

    def _hist(self, values: np.ndarray) -> DataArray:
        dim = self._dim
        return DataArray(values.reshape(-1), (dim,), 'counts',
                         {dim: Variable((dim,), self._coord, self._edges.unit)})

    def _finalize_histogram_mode(self) -> dict[str, Any]:
        if not self._hdata:
            raise ValueError('No data has been added')
        cur = self._hcur.cpu().numpy()
        cum = self._hcum.cpu().numpy()
        self._hcur.zero_()
        self._hdata = False
        dim = 'time_of_arrival'
        coord = Variable((dim,), np.asarray(self._edges.get_edges(), dtype=np.float64),
                         self._edges.unit)
        lo, hi = self._hslice

        def h(v):
            return DataArray(v, (dim,), 'counts', {dim: coord})

        def scalar(x):
            return DataArray(np.asarray(float(x)), (), 'counts')

        return {
            'cumulative': h(cum),
            'current': h(cur),
            'counts_total': scalar(cur.sum()),
            'counts_in_toa_range': scalar(cur[lo:hi].sum()),
            'counts_total_cumulative': scalar(cum.sum()),
            'counts_in_toa_range_cumulative': scalar(cum[lo:hi].sum()),
        }

    def finalize(self) -> dict[str, Any]:
        if self._hist_mode:
            out = self._finalize_histogram_mode()
            _stamp_window(out, MONITOR_WINDOW_OUTPUTS, self._start, self._end)
            self._start = self._end = None
            return publish(out)
        res = self._engine.finalize(images=False, hists=True)
        out = {
            'cumulative': self._hist(res.cumulative_hist),
            'current': self._hist(res.current_hist),
            'counts_total': DataArray(np.asarray(float(res.current_total)), (), 'counts'),
            'counts_in_toa_range': DataArray(np.asarray(float(res.current_in_range)), (), 'counts'),
            'counts_total_cumulative': DataArray(np.asarray(float(res.cumulative_total)), (), 'counts'),
            'counts_in_toa_range_cumulative': DataArray(
                np.asarray(float(res.cumulative_in_range)), (), 'counts'
            ),
        }
        _stamp_window(out, MONITOR_WINDOW_OUTPUTS, self._start, self._end)
        self._start = self._end = None
        return publish(out)

    def clear(self) -> None:
        self._engine.clear()
        if self._hcur is not None:
            self._hcur.zero_()
            self._hcum.zero_()
        self._hdata = False
        self._start = self._end = None


def create_gpu_monitor_workflow(source_name: str, edges, *,
                                range_filter: tuple[float, float] | None = None,
                                coordinate_mode: str = 'toa',
                                lookup_table: 'WavelengthLookupTable | None' = None,
                                monitor_distance: float | None = None,
                                device: int = 0) -> GpuMonitorWorkflow:
    """``create_monitor_workflow`` (monitor_workflow.py:225-331); the lookup
    table and the monitor's Ltotal stand for its ``lookup_table_filename`` and
    ``geometry_filename``."""
    return GpuMonitorWorkflow(source_name, edges, range_filter=range_filter,
                              coordinate_mode=coordinate_mode, lookup_table=lookup_table,
                              monitor_distance=monitor_distance, device=device)
