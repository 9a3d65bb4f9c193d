"""Synthetic instrument shapes and ev44-like event streams.

No geometry files or recorded streams are available offline, so benchmark and
test inputs are generated here with fixed seeds.  Shapes and distributions
follow the reference's instrument configs and fakes:

* dummy ``panel_0``: pids 1..16384 (dummy/streams.py:11), identity logical view
  128 x 128 (dummy/factories.py:40-51); TOA ``uniform(0, 70e6)``
  (tests/helpers/livedata_app.py:189) or ``normal(30e6, 1e7)``
  (services/fake_detectors.py:98-99, 142-145).
* LOKI bank 0: pids 1..802816 (loki/streams.py:18), xy_plane 144 x 144
  (loki/factories.py:101-121); TOA ``uniform(0, 71e6)``.  Banks 1-8
  (``loki_bank``): the window-frame panels with their pid ranges and
  resolutions (loki/streams.py:17-27, loki/factories.py:101-112).
* DREAM mantle: pids 229377..720896 (dream/streams.py:19), cylinder_mantle_z
  80 x 320 (dream/factories.py:59-66), sigma 4 mm noise, 4 noisy replicas + the
  original; Zipf(1.2) pixel skew over a random permutation; TOA 80 % normal(30 ms,
  10 ms) + 20 % in 3 hot bins; ``geomspace(0.5, 71.43, 101)`` ms edges.
* BIFROST unified detector: pids 1..13500 folded (arc 5, tube 3, channel 9,
  pixel 100) (bifrost/streams.py:46-48), logical 15 x 900, float32.

Geometric views start from synthetic calibrated pixel positions and go
through the restated essreduce projections and noise replicas
(``geometry.GeometricSource``); ``Instrument.coords`` holds the projected
per-replica coordinates the LUT is built from.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .edges import ESS_PULSE_PERIOD_MS, TOAEdges


@dataclass
class Instrument:
    name: str
    detector_number: np.ndarray
    coords: dict[str, np.ndarray] | None  # (R, P) per screen dim, geometric views
    resolution: dict[str, int] | None
    edges: TOAEdges
    out_dtype: str = 'float64'
    positions: np.ndarray | None = None  # (P, 3) calibrated pixel positions (m)
    projection_type: str | None = None
    pixel_noise: object = None


def dream_mantle(n_replicas: int = 5, seed: int = 7) -> Instrument:
    """DREAM mantle: 1280 x 384 pixels on a cylinder of radius 1.1 m about the
    beam (z) axis, projected with the restated ``cylinder_mantle_z`` and sigma
    = 4 mm gaussian noise replicas (dream/factories.py:56-66) through
    ``geometry.GeometricSource``."""
    from .geometry import GeometricSource, PixelNoise

    first, last = 229377, 720896
    n_phi, n_z = 1280, 384
    phi = np.linspace(-2.4, 2.4, n_phi)
    zz = np.linspace(-0.8, 0.8, n_z)
    pp, zz2 = np.meshgrid(phi, zz, indexing='ij')
    radius = 1.1
    pos = np.stack([radius * np.cos(pp).ravel(), radius * np.sin(pp).ravel(), zz2.ravel()], -1)
    dn = np.arange(first, last + 1, dtype=np.int32)
    res = {'arc_length': 80, 'z': 320}
    noise = PixelNoise(sigma=0.004, replicas=n_replicas - 1, seed=seed) if n_replicas > 1 else None
    src = GeometricSource(dn, pos, projection_type='cylinder_mantle_z', resolution=res,
                          pixel_noise=noise)
    return Instrument(
        name='dream_mantle',
        detector_number=dn,
        coords=src.coords(),
        resolution=res,
        edges=TOAEdges(start=0.5, stop=ESS_PULSE_PERIOD_MS, num_bins=100, scale='log'),
        positions=pos,
        projection_type='cylinder_mantle_z',
        pixel_noise=noise,
    )


DREAM_L1 = 76.55  # m, source -> sample


def dream_wavelength_table(distance_min: float = 77.5, distance_max: float = 78.1):
    """Direct-flight wavelength table covering DREAM mantle flight paths
    (Ltotal 77.65..77.91 m): 0.05 m x 0.25 ms grid over one pulse period."""
    from .wavelength import ideal_lookup_table

    n_d = int(round((distance_max - distance_min) / 0.05)) + 1
    return ideal_lookup_table(distance_min, distance_max, n_d, 71.5e6, 287)


# LOKI's nine detector banks: pixel-id ranges (config/instruments/loki/streams.py:
# 17-27) and xy_plane resolutions (loki/factories.py:101-112)
LOKI_BANKS: dict[str, tuple[int, int]] = {
    'loki_detector_0': (1, 802816),
    'loki_detector_1': (802817, 1032192),
    'loki_detector_2': (1032193, 1204224),
    'loki_detector_3': (1204225, 1433600),
    'loki_detector_4': (1433601, 1605632),
    'loki_detector_5': (1605633, 2007040),
    'loki_detector_6': (2007041, 2465792),
    'loki_detector_7': (2465793, 2752512),
    'loki_detector_8': (2752513, 3211264),
}
LOKI_RESOLUTIONS: dict[str, dict[str, int]] = {
    'loki_detector_0': {'y': 144, 'x': 144},
    **{f'loki_detector_{b}': ({'y': 36, 'x': 108} if b % 2 else {'y': 108, 'x': 36})
       for b in range(1, 9)},
}


def loki_bank(bank: int, n_replicas: int = 5, seed: int = 42) -> Instrument:
    """LOKI bank ``bank``: bank 0 is :func:`loki_bank0`; banks 1-8 are the two
    window frames (z = 3.5 m and 1.5 m) of 448-pixel-wide panels, the odd banks above / below the beam (wide, 36 x
    108 screens), the even ones left / right of it (tall, 108 x 36).  Projected
    with the restated ``xy_plane`` and cylindrical-pixel noise replicas
    (loki/factories.py:101-121: straw pixels along x, flip_x)."""
    from .geometry import GeometricSource, PixelNoise

    if bank == 0:
        return loki_bank0(n_replicas, seed)
    name = f'loki_detector_{bank}'
    first, last = LOKI_BANKS[name]
    p = last - first + 1
    n_long = p // 448
    frame = (bank - 1) // 4          # 0: first window frame, 1: second
    side = (bank - 1) % 4            # above, left, below, right of the beam
    z = 3.5 if frame == 0 else 1.5
    off = 0.7 if frame == 0 else 0.9
    if bank % 2:                     # wide: straws along x
        nx, ny = n_long, 448
        x0, y0 = 0.0, off if side == 0 else -off
    else:                            # tall
        nx, ny = 448, n_long
        x0, y0 = -off if side == 1 else off, 0.0
    w = 0.6
    xs = x0 + np.linspace(-w / 2, w / 2, nx)
    ys = y0 + np.linspace(-w / 2, w / 2, ny) * (ny / max(nx, ny))
    xx, yy = np.meshgrid(xs, ys, indexing='xy')
    pos = np.stack([xx.ravel(), yy.ravel(), np.full(p, z)], -1)
    dn = np.arange(first, last + 1, dtype=np.int32)
    res = dict(LOKI_RESOLUTIONS[name])
    dx = w / max(nx - 1, 1)
    noise = (PixelNoise(cylinder_axis=(dx, 0.0, 0.0), cylinder_radius=dx / 2,
                        replicas=n_replicas - 1, seed=seed + bank) if n_replicas > 1 else None)
    src = GeometricSource(dn, pos, projection_type='xy_plane', resolution=res, pixel_noise=noise)
    return Instrument(
        name=name,
        detector_number=dn,
        coords=src.coords(),
        resolution=res,
        edges=TOAEdges(),
        positions=pos,
        projection_type='xy_plane',
        pixel_noise=noise,
    )


def loki_bank0(n_replicas: int = 5, seed: int = 42) -> Instrument:
    """LOKI bank 0: 896 x 896 pixels on a plane 5 m downstream, projected with
    the restated ``xy_plane`` and cylindrical-pixel noise replicas
    (loki/factories.py:101-121: straw pixels along x)."""
    from .geometry import GeometricSource, PixelNoise

    p = 802816
    side = 896
    xs = np.linspace(-0.5, 0.5, side)
    xx, yy = np.meshgrid(xs, xs, indexing='ij')
    pos = np.stack([xx.ravel(), yy.ravel(), np.full(p, 5.0)], -1)
    dn = np.arange(1, p + 1, dtype=np.int32)
    res = {'y': 144, 'x': 144}
    noise = (PixelNoise(cylinder_axis=(1.0 / side, 0.0, 0.0), cylinder_radius=0.5 / side,
                        replicas=n_replicas - 1, seed=seed) if n_replicas > 1 else None)
    src = GeometricSource(dn, pos, projection_type='xy_plane', resolution=res, pixel_noise=noise)
    return Instrument(
        name='loki_bank0',
        detector_number=dn,
        coords=src.coords(),
        resolution=res,
        edges=TOAEdges(),
        positions=pos,
        projection_type='xy_plane',
        pixel_noise=noise,
    )


def dummy_panel() -> Instrument:
    return Instrument(
        name='dummy',
        detector_number=np.arange(1, 128**2 + 1, dtype=np.int32).reshape(128, 128),
        coords=None,
        resolution=None,
        edges=TOAEdges(),
    )


def bifrost_unified() -> Instrument:
    return Instrument(
        name='bifrost',
        detector_number=np.arange(1, 5 * 3 * 9 * 100 + 1, dtype=np.int32).reshape(5, 3, 9, 100),
        coords=None,
        resolution=None,
        edges=TOAEdges(),
        out_dtype='float32',
    )


def bifrost_transform(idx: np.ndarray) -> np.ndarray:
    """``_logical_view`` (bifrost/specs.py:285-299): flatten (arc, tube) and
    (channel, pixel) -> (15, 900)."""
    return idx.reshape(15, 900)


# ---------------------------------------------------------------------------
# logical views over folded banks (DREAM, MAGIC)
# ---------------------------------------------------------------------------
# Logical voxel structure of the DREAM banks, ``ess.dream.workflows.
# DETECTOR_BANK_SIZES`` (essreduce-side package, not in /root/reference;
# the mantle's dim order is the one dream/views.py:47-48 states: after the
# fold the dims are (wire, module, segment, strip, counter)).  The mantle's
# product is its 491,520 pixels (dream/streams.py:19).
DREAM_BANK_SIZES: dict[str, dict[str, int]] = {
    'mantle_detector': {'wire': 32, 'module': 5, 'segment': 6, 'strip': 256, 'counter': 2},
}

# MAGIC banks, as the reference defines them (magic/views.py:32-35).
MAGIC_BANK_SIZES: dict[str, dict[str, int]] = {
    'magic_detector_a': {'wire': 32, 'strip': 128, 'segment': 120},
    'magic_detector_b': {'wire': 32, 'strip': 16, 'segment': 256},
}


def dream_mantle_front_layer(da, source_name: str):
    """``get_mantle_front_layer`` (dream/views.py:13-21): wire 0 only,
    (mod/seg/cntr, strip)."""
    return (
        da.fold(dim=da.dim, sizes=DREAM_BANK_SIZES[source_name])
        .transpose(('wire', 'module', 'segment', 'counter', 'strip'))['wire', 0]
        .flatten(('module', 'segment', 'counter'), to='mod/seg/cntr')
    )


def dream_wire_view(da, source_name: str):
    """``get_wire_view`` (dream/views.py:24-53): (strip, wire, mod/seg/cntr);
    the view reduces ``strip``."""
    return (
        da.fold(dim=da.dim, sizes=DREAM_BANK_SIZES[source_name])
        .transpose(('strip', 'wire', 'module', 'segment', 'counter'))
        .flatten(('module', 'segment', 'counter'), to='mod/seg/cntr')
    )


def dream_strip_view(da, source_name: str):
    """``get_strip_view`` (dream/views.py:56-85): (other, strip); the view
    reduces ``other``."""
    folded = da.fold(dim=da.dim, sizes=DREAM_BANK_SIZES[source_name])
    rest = tuple(d for d in folded.dims if d != 'strip')
    if len(rest) > 1:
        folded = folded.transpose((*rest, 'strip')).flatten(rest, to='other')
    return folded


def magic_wire_view(da, source_name: str):
    """``get_wire_view`` (magic/views.py:38-58): (wire, strip, segment); the
    view reduces ``strip``."""
    return da.fold(dim=da.dim, sizes=MAGIC_BANK_SIZES[source_name])


def magic_strip_view(da, source_name: str):
    """``get_strip_view`` (magic/views.py:61-85): (wire/segment, strip); the
    view reduces ``wire/segment``."""
    folded = da.fold(dim=da.dim, sizes=MAGIC_BANK_SIZES[source_name])
    return folded.transpose(('wire', 'segment', 'strip')).flatten(('wire', 'segment'),
                                                                   to='wire/segment')


def dream_logical_views() -> dict:
    """The DREAM logical views registered for the mantle (dream/specs.py:
    151-180): name -> ``LogicalViewConfig``."""
    from .workflows import LogicalViewConfig

    return {
        'mantle_front_layer': LogicalViewConfig(transform=dream_mantle_front_layer),
        'wire_view': LogicalViewConfig(transform=dream_wire_view, roi_support=False,
                                       reduction_dim='strip'),
        'strip_view': LogicalViewConfig(transform=dream_strip_view, roi_support=False,
                                        reduction_dim='other'),
    }


def magic_logical_views() -> dict:
    """MAGIC's wire and strip views (magic/specs.py:93-111)."""
    from .workflows import LogicalViewConfig

    return {
        'wire_view': LogicalViewConfig(transform=magic_wire_view, roi_support=False,
                                       reduction_dim='strip'),
        'strip_view': LogicalViewConfig(transform=magic_strip_view, roi_support=False,
                                        reduction_dim='wire/segment'),
    }


def magic_bank(name: str = 'magic_detector_a', first: int = 1) -> Instrument:
    """A MAGIC bank: contiguous detector numbers over its voxels."""
    n = int(np.prod(list(MAGIC_BANK_SIZES[name].values())))
    return Instrument(name=name, detector_number=np.arange(first, first + n, dtype=np.int32),
                      coords=None, resolution=None, edges=TOAEdges())


# ---------------------------------------------------------------------------
# event streams (numpy, for tests and the CPU baseline)
# ---------------------------------------------------------------------------
def zipf_pixel_weights(p: int, s: float = 1.2, seed: int = 7) -> np.ndarray:
    rng = np.random.default_rng(seed + 1000)
    w = np.arange(1, p + 1, dtype=np.float64) ** (-s)
    w = w[rng.permutation(p)]
    return w / w.sum()


def dream_hot_bins(edges_ns: np.ndarray) -> list[tuple[float, float]]:
    # bins 40, 62 and 85 of 100: the same fractions of the edge list for any
    # bin count, so the peaks stay at the same times when the edges share
    # start, stop and scale
    nb = len(edges_ns) - 1
    return [(edges_ns[b], edges_ns[b + 1]) for b in (40 * nb // 100, 62 * nb // 100, 85 * nb // 100)]


def with_toa_edges(inst: Instrument, num_bins: int | None = None, scale: str | None = None,
                   start: float | None = None) -> Instrument:
    """The instrument with other TOA edges (any ``EdgesModel`` configuration:
    1..10000 bins, linear or log, parameter_models.py:82-105)."""
    import dataclasses

    e = inst.edges
    edges = dataclasses.replace(e, num_bins=num_bins or e.num_bins, scale=scale or e.scale,
                                start=e.start if start is None else start)
    return dataclasses.replace(inst, edges=edges)


def dream_events(n: int, inst: Instrument, seed: int = 7, cdf: np.ndarray | None = None):
    rng = np.random.default_rng(seed)
    dn = inst.detector_number.ravel()
    if cdf is None:
        cdf = np.cumsum(zipf_pixel_weights(len(dn)))
    pix = np.minimum(np.searchsorted(cdf, rng.random(n)), len(dn) - 1)
    pid = dn[pix].astype(np.int32)
    edges = inst.edges.edges_ns()
    toa = rng.normal(30e6, 10e6, n)
    hot = rng.random(n) < 0.2
    which = rng.integers(0, 3, n)
    hb = np.array(dream_hot_bins(edges))
    lo, hi = hb[which, 0], hb[which, 1]
    toa = np.where(hot, lo + rng.random(n) * (hi - lo), toa)
    return pid, toa.astype(np.int32)


def uniform_events(n: int, first: int, last: int, seed: int = 42, toa_max: float = 71e6):
    rng = np.random.default_rng(seed)
    pid = rng.integers(first, last + 1, n, dtype=np.int64).astype(np.int32)
    toa = rng.uniform(0, toa_max, n).astype(np.int32)
    return pid, toa


def fake_detector_events(n: int, first: int, last: int, seed: int = 1234):
    """fake_detectors.py:98-103: normal(30e6, 1e7) TOA, uniform pixel ids."""
    rng = np.random.default_rng(seed)
    toa = rng.normal(loc=30_000_000, scale=10_000_000, size=n).astype(np.int64).astype(np.int32)
    pid = rng.integers(low=first, high=last + 1, size=n).astype(np.int32)
    return pid, toa


# ---------------------------------------------------------------------------
# device-side generators (torch, for the benchmark: inputs resident in HBM)
# ---------------------------------------------------------------------------
def torch_dream_events(n: int, inst: Instrument, seed: int, device):
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    dn = torch.as_tensor(inst.detector_number.ravel(), device=device)
    cdf = torch.as_tensor(np.cumsum(zipf_pixel_weights(len(dn))), device=device)
    u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    pix = torch.clamp(torch.searchsorted(cdf, u), max=len(dn) - 1)
    pid = dn[pix].to(torch.int32)
    del pix, u
    edges = inst.edges.edges_ns()
    toa = torch.randn(n, generator=g, device=device, dtype=torch.float32) * 10e6 + 30e6
    hot = torch.rand(n, generator=g, device=device) < 0.2
    which = torch.randint(0, 3, (n,), generator=g, device=device)
    hb = torch.as_tensor(np.array(dream_hot_bins(edges)), device=device, dtype=torch.float64)
    lo, hi = hb[which, 0], hb[which, 1]
    hot_toa = lo + torch.rand(n, generator=g, device=device, dtype=torch.float64) * (hi - lo)
    toa = torch.where(hot, hot_toa, toa.to(torch.float64)).to(torch.int32)
    return pid.contiguous(), toa.contiguous()


def torch_uniform_events(n: int, first: int, last: int, seed: int, device, toa_max: float = 71e6):
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    pid = torch.randint(first, last + 1, (n,), generator=g, device=device, dtype=torch.int32)
    toa = (torch.rand(n, generator=g, device=device, dtype=torch.float64) * toa_max).to(
        torch.int32
    )
    return pid.contiguous(), toa.contiguous()


def bifrost_spectrum_config(pixels_per_tube: int = 10):
    """BIFROST ``spectrum_view`` (bifrost/specs.py:311-349) in index form: the
    (15, 900) screen folded to (arc 5, tube 3, channel 9, pixel, subpixel),
    subpixel summed, (tube, channel, pixel) flattened -> (arc, detector_number)."""
    from .workflows import SpectrumViewConfig

    if 100 % pixels_per_tube:
        raise ValueError('pixels_per_tube must divide 100')
    sub = 100 // pixels_per_tube

    def transform(idx: np.ndarray) -> np.ndarray:
        return idx.reshape(5, 3, 9, pixels_per_tube, sub).reshape(5, 3 * 9 * pixels_per_tube, sub)

    return SpectrumViewConfig(transform=transform, output_dims=('arc', 'detector_number'),
                              reduction_axes=(2,))
