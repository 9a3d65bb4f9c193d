"""Geometry -> LUT builder for geometric detector views.

Setup-time host code: from calibrated pixel positions to the per-replica
projected screen coordinates the engine's LUT is built from, then to the LUT
itself (``projection.geometric_lut``).  Restated from the published algorithm
of essreduce 26.6.3 ``ess.reduce.live.raw`` (not vendored under
/root/reference and not installed here), as the reference calls it:

* replicas: ``position_with_noisy_replicas`` -- replica 0 is the calibrated
  position itself, replicas 1..R are ``position + noise`` with
  ``PositionNoiseReplicaCount = 4`` (SRC/workflows/detector_view/workflow.py:
  180-198);
* noise: ``gaussian_position_noise`` (isotropic, sigma per component; DREAM
  sigma = 4 mm, SRC/config/instruments/dream/factories.py:59) or
  ``position_noise_for_cylindrical_pixel`` (uniform inside the pixel's
  cylinder; LOKI ``pixel_noise='cylindrical'``, loki/factories.py:120);
* projections (SRC/workflows/detector_view/projectors.py:306-352):
  ``make_xy_plane_coords`` -- every point is moved along its ray from the
  sample (origin) onto the plane z = min(z), giving screen ``x``, ``y``;
  ``make_cylinder_mantle_coords(axis)`` -- along the ray onto the cylinder
  about ``axis`` through the origin whose radius is the smallest radial
  distance of any point, giving ``arc_length = radius * phi`` and the axial
  coordinate;
* ``flip_x`` and the scipp edge rule are applied by ``geometric_lut``
  (projectors.py:341-350).

Parity: the projection formulas are a restatement of essreduce's published
code (parity unpinned: essreduce is absent offline); the noise draws use
numpy's generator with a caller seed, so noisy replicas are not bit-equal to
essreduce's (parity unpinned).  Everything downstream of the
projected coordinates is pinned (tests/test_geometry.py; the flip_x KAT of
tests/workflows/detector_view/projectors_test.py:140-178 passes through
``make_xy_plane_coords``).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .projection import ViewLUT, geometric_lut

POSITION_NOISE_REPLICA_COUNT = 4  # detector_view/workflow.py:187, 193
NOISE_POOL = 1_000_000  # noise vectors drawn once, sampled per (replica, pixel)
PROJECTIONS = ('xy_plane', 'cylinder_mantle_y', 'cylinder_mantle_z')


def _vec(a) -> np.ndarray:
    v = np.asarray(a, dtype=np.float64)
    if v.shape[-1] != 3:
        raise ValueError(f'positions must have a trailing dimension of 3, got {v.shape}')
    return v


# ---------------------------------------------------------------------------
# noise
# ---------------------------------------------------------------------------
def gaussian_position_noise(sigma: float, *, size: int = NOISE_POOL, seed: int = 0) -> np.ndarray:
    """``gaussian_position_noise``: ``(size, 3)`` isotropic normal offsets (m)."""
    if sigma < 0:
        raise ValueError('sigma must be >= 0')
    return np.random.default_rng(seed).normal(0.0, float(sigma), size=(size, 3))


def position_noise_for_cylindrical_pixel(axis, radius: float, *, size: int = NOISE_POOL,
                                         seed: int = 0) -> np.ndarray:
    """``position_noise_for_cylindrical_pixel``: ``(size, 3)`` offsets uniform
    inside a cylinder of ``radius`` whose axis vector ``axis`` spans the pixel
    (offsets along it uniform in [-1/2, 1/2] of its length, radially uniform
    over the disk: r = radius * sqrt(u))."""
    ax = _vec(axis).reshape(3)
    length = float(np.linalg.norm(ax))
    if length == 0 or radius < 0:
        raise ValueError('pixel cylinder needs a non-zero axis and radius >= 0')
    u = ax / length
    # orthonormal basis of the plane normal to the axis
    helper = np.array([1.0, 0.0, 0.0]) if abs(u[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
    e1 = np.cross(u, helper)
    e1 /= np.linalg.norm(e1)
    e2 = np.cross(u, e1)
    rng = np.random.default_rng(seed)
    along = rng.uniform(-0.5, 0.5, size) * length
    r = float(radius) * np.sqrt(rng.uniform(0.0, 1.0, size))
    phi = rng.uniform(0.0, 2.0 * np.pi, size)
    return (along[:, None] * u + (r * np.cos(phi))[:, None] * e1
            + (r * np.sin(phi))[:, None] * e2)


def position_with_noisy_replicas(position, noise: np.ndarray | None, *,
                                 replicas: int = POSITION_NOISE_REPLICA_COUNT,
                                 seed: int = 0) -> np.ndarray:
    """``position_with_noisy_replicas``: ``(1 + replicas, P, 3)``; replica 0 is
    ``position``, replica k >= 1 is ``position`` plus noise vectors drawn from
    the pool.  ``noise=None`` or ``replicas=0`` gives the position alone."""
    pos = _vec(position).reshape(-1, 3)
    if noise is None or replicas <= 0:
        return pos[None]
    pool = _vec(noise).reshape(-1, 3)
    rng = np.random.default_rng(seed + 1)
    idx = rng.integers(0, len(pool), size=(replicas, len(pos)))
    return np.concatenate([pos[None], pos[None] + pool[idx]], axis=0)


# ---------------------------------------------------------------------------
# projections
# ---------------------------------------------------------------------------
def make_xy_plane_coords(position) -> dict[str, np.ndarray]:
    """``make_xy_plane_coords``: ``{'x', 'y'}`` of shape ``(R, P)``, each point
    moved along its ray from the origin onto the plane ``z = min(z)``."""
    p = _vec(position)
    if p.ndim == 2:
        p = p[None]
    z = p[..., 2]
    zplane = float(np.nanmin(z))
    if zplane == 0.0 or np.any(np.sign(z[np.isfinite(z)]) != np.sign(zplane)):
        raise ValueError('xy_plane projection needs every pixel on one side of z = 0')
    t = zplane / z
    return {'x': p[..., 0] * t, 'y': p[..., 1] * t}


def make_cylinder_mantle_coords(position, axis: str = 'z') -> dict[str, np.ndarray]:
    """``make_cylinder_mantle_coords(axis)``: ``{'arc_length', axis}`` of shape
    ``(R, P)``, each point moved along its ray from the origin onto the
    cylinder about ``axis`` with the smallest radial distance as radius;
    ``arc_length = radius * phi``, phi measured as atan2(y, x) about z and
    atan2(x, z) about y."""
    p = _vec(position)
    if p.ndim == 2:
        p = p[None]
    x, y, z = p[..., 0], p[..., 1], p[..., 2]
    if axis == 'z':
        a, b, along = x, y, z
    elif axis == 'y':
        a, b, along = z, x, y
    else:
        raise ValueError(f'cylinder axis must be "y" or "z", got {axis!r}')
    r = np.hypot(a, b)
    radius = float(np.nanmin(r))
    if not radius > 0:
        raise ValueError('cylinder projection needs every pixel off the axis')
    t = radius / r
    phi = np.arctan2(b, a)
    return {'arc_length': radius * phi, axis: along * t}


def project(position, projection_type: str) -> dict[str, np.ndarray]:
    if projection_type == 'xy_plane':
        return make_xy_plane_coords(position)
    if projection_type in ('cylinder_mantle_y', 'cylinder_mantle_z'):
        return make_cylinder_mantle_coords(position, axis=projection_type[-1])
    raise ValueError(f'Unknown projection type: {projection_type}')


# ---------------------------------------------------------------------------
# detector transform (the geometry signal of geometry_signal.py:27-51)
# ---------------------------------------------------------------------------
def apply_transform(transform, offsets) -> np.ndarray:
    """Pixel positions of a rigid component: ``transform`` is a 3-vector
    (translation), a 3x3 matrix (linear) or a 4x4 affine matrix, applied to
    the pixel offsets in the component's frame."""
    off = _vec(offsets).reshape(-1, 3)
    if transform is None:
        return off.copy()
    t = np.asarray(transform, dtype=np.float64)
    if t.shape == (3,):
        return off + t
    if t.shape == (3, 3):
        return off @ t.T
    if t.shape == (4, 4):
        return off @ t[:3, :3].T + t[:3, 3]
    raise ValueError(f'unsupported transform shape {t.shape}')


@dataclass
class PixelNoise:
    """``pixel_noise`` of ``GeometricViewConfig``: ``sigma`` (gaussian, m) or a
    cylindrical pixel (``axis`` vector spanning the pixel, ``radius``)."""

    sigma: float | None = None
    cylinder_axis: tuple[float, float, float] | None = None
    cylinder_radius: float | None = None
    replicas: int = POSITION_NOISE_REPLICA_COUNT
    seed: int = 0

    def pool(self) -> np.ndarray:
        if self.sigma is not None:
            return gaussian_position_noise(self.sigma, seed=self.seed)
        if self.cylinder_axis is not None and self.cylinder_radius is not None:
            return position_noise_for_cylindrical_pixel(self.cylinder_axis, self.cylinder_radius,
                                                        seed=self.seed)
        raise ValueError('PixelNoise needs sigma or cylinder_axis + cylinder_radius')


def noise_from_config(pixel_noise, pixel_shape: dict | None = None) -> PixelNoise | None:
    """Map the reference's ``pixel_noise`` (None, ``'cylindrical'``, or a sigma
    in m) onto :class:`PixelNoise`; ``'cylindrical'`` takes the pixel's
    cylinder from ``pixel_shape`` ({'axis': (3,), 'radius': float}), which the
    reference reads from the NeXus pixel_shape."""
    if pixel_noise is None:
        return None
    if isinstance(pixel_noise, PixelNoise):
        return pixel_noise
    if isinstance(pixel_noise, str):
        if pixel_noise != 'cylindrical':
            raise ValueError(f'Invalid pixel_noise: {pixel_noise}')
        if not pixel_shape:
            raise ValueError("pixel_noise='cylindrical' needs the pixel shape (axis, radius)")
        return PixelNoise(cylinder_axis=tuple(pixel_shape['axis']),
                          cylinder_radius=float(pixel_shape['radius']))
    return PixelNoise(sigma=float(pixel_noise))


class GeometricSource:
    """A geometric view's geometry: pixel offsets in the component frame, the
    projection and noise config; builds the view LUT for a given component
    transform (and rebuilds it when the transform changes).  The noisy
    replicas are drawn once and move rigidly with the component."""

    def __init__(self, detector_number, offsets, *, projection_type: str,
                 resolution: dict[str, int], pixel_noise=None, flip_x: bool = False,
                 pixel_shape: dict | None = None, transform=None) -> None:
        if projection_type not in PROJECTIONS:
            raise ValueError(f'Unknown projection type: {projection_type}')
        self.detector_number = np.asarray(detector_number)
        off = _vec(offsets).reshape(-1, 3)
        if len(off) != self.detector_number.size:
            raise ValueError(f'{len(off)} pixel positions for {self.detector_number.size} pixels')
        self.projection_type = projection_type
        self.resolution = dict(resolution)
        self.flip_x = bool(flip_x)
        noise = noise_from_config(pixel_noise, pixel_shape)
        self.local = (position_with_noisy_replicas(off, noise.pool(), replicas=noise.replicas,
                                                   seed=noise.seed)
                      if noise is not None else off[None])
        self.transform = transform

    @property
    def n_replicas(self) -> int:
        return self.local.shape[0]

    def positions(self, transform=None) -> np.ndarray:
        t = self.transform if transform is None else transform
        r, p, _ = self.local.shape
        return apply_transform(t, self.local.reshape(-1, 3)).reshape(r, p, 3)

    def pixel_positions(self, transform=None) -> np.ndarray:
        """Noise-free pixel positions (replica 0), ``(P, 3)``."""
        t = self.transform if transform is None else transform
        return apply_transform(t, self.local[0])

    def coords(self, transform=None) -> dict[str, np.ndarray]:
        return project(self.positions(transform), self.projection_type)

    def view(self, transform=None) -> ViewLUT:
        return geometric_lut(self.detector_number, self.coords(transform), self.resolution,
                             flip_x=self.flip_x)
