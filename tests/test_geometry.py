"""Geometry -> LUT builder (esslivedata_amd/geometry.py), CPU.

The projection formulas restate essreduce's ``ess.reduce.live.raw`` (absent
offline: parity unpinned beyond the reference KATs); these tests pin the
geometric properties the restatement promises and the LUT it feeds.
"""

import numpy as np
import pytest

from esslivedata_amd import geometry, projection


def test_xy_plane_moves_points_along_rays_onto_nearest_plane():
    pos = np.array([[0.1, 0.2, 2.0], [0.4, -0.2, 4.0], [-1.0, 0.0, 2.0]])
    c = geometry.make_xy_plane_coords(pos)
    np.testing.assert_allclose(c['x'][0], [0.1, 0.2, -1.0])
    np.testing.assert_allclose(c['y'][0], [0.2, -0.1, 0.0])
    with pytest.raises(ValueError):
        geometry.make_xy_plane_coords(np.array([[0, 0, 1.0], [0, 0, -1.0]]))


@pytest.mark.parametrize('axis', ['z', 'y'])
def test_cylinder_mantle_arc_length_and_axial_coordinate(axis):
    phi = np.linspace(-2.0, 2.0, 9)
    r = np.array([1.0, 2.0, 1.0, 1.5, 1.0, 1.0, 3.0, 1.0, 1.0])
    h = np.linspace(-0.5, 0.5, 9)
    if axis == 'z':
        pos = np.stack([r * np.cos(phi), r * np.sin(phi), h * r], -1)
    else:  # about y: phi measured from z towards x
        pos = np.stack([r * np.sin(phi), h * r, r * np.cos(phi)], -1)
    c = geometry.make_cylinder_mantle_coords(pos, axis=axis)
    np.testing.assert_allclose(c['arc_length'][0], 1.0 * phi, atol=1e-12)
    # along the ray onto the radius-1 cylinder: the axial coordinate scales by 1 / r
    np.testing.assert_allclose(c[axis][0], h, atol=1e-12)
    with pytest.raises(ValueError):
        geometry.make_cylinder_mantle_coords(pos, axis='x')


def test_noise_replicas():
    pos = np.random.default_rng(0).normal(size=(1000, 3))
    g = geometry.gaussian_position_noise(0.004, seed=3)
    rep = geometry.position_with_noisy_replicas(pos, g, replicas=4)
    assert rep.shape == (5, 1000, 3)
    np.testing.assert_array_equal(rep[0], pos)  # replica 0 = calibrated position
    d = rep[1:] - pos
    assert abs(d.std() - 0.004) < 2e-4 and not np.array_equal(rep[1], rep[2])
    axis, radius = (0.0, 0.0, 0.01), 0.002
    cyl = geometry.position_noise_for_cylindrical_pixel(axis, radius, seed=5)
    assert np.all(np.abs(cyl[:, 2]) <= 0.005 + 1e-15)
    assert np.all(np.hypot(cyl[:, 0], cyl[:, 1]) <= radius + 1e-15)
    # uniform over the disk: half the points inside radius / sqrt(2)
    frac = np.mean(np.hypot(cyl[:, 0], cyl[:, 1]) < radius / np.sqrt(2))
    assert abs(frac - 0.5) < 0.01
    assert geometry.position_with_noisy_replicas(pos, None).shape == (1, 1000, 3)


def test_noise_from_config_matches_reference_options():
    assert geometry.noise_from_config(None) is None
    assert geometry.noise_from_config(0.004).sigma == 0.004
    n = geometry.noise_from_config('cylindrical', {'axis': (0, 0, 0.01), 'radius': 0.004})
    assert n.cylinder_radius == 0.004 and n.replicas == 4
    with pytest.raises(ValueError):
        geometry.noise_from_config('cylindrical')
    with pytest.raises(ValueError):
        geometry.noise_from_config('spherical')


def test_transform_and_rebuild():
    dn = np.arange(100, 112, dtype=np.int32)
    off = np.stack([np.linspace(-0.1, 0.1, 12), np.linspace(-0.05, 0.05, 12), np.zeros(12)], -1)
    src = geometry.GeometricSource(dn, off, projection_type='xy_plane',
                                   resolution={'x': 4, 'y': 3}, transform=(0.0, 0.0, 2.0))
    v0 = src.view()
    exp = projection.geometric_lut(dn, geometry.make_xy_plane_coords(off + [0, 0, 2.0]),
                                   {'x': 4, 'y': 3})
    np.testing.assert_array_equal(v0.lut, exp.lut)
    # a 90-degree rotation about z swaps the roles of x and y
    rot = np.eye(4)
    rot[:3, :3] = [[0, -1, 0], [1, 0, 0], [0, 0, 1]]
    rot[2, 3] = 2.0
    v1 = src.view(rot)
    assert v1.lut.shape == v0.lut.shape and not np.array_equal(v1.lut, v0.lut)
    np.testing.assert_allclose(src.positions(rot)[0][:, 0], -off[:, 1])
    with pytest.raises(ValueError):
        geometry.apply_transform(np.eye(2), off)


def test_synthetic_instruments_use_the_builder():
    from esslivedata_amd import synthetic

    inst = synthetic.dream_mantle()
    assert inst.coords['arc_length'].shape == (5, 491520)
    src = geometry.GeometricSource(inst.detector_number, inst.positions,
                                   projection_type=inst.projection_type,
                                   resolution=inst.resolution, pixel_noise=inst.pixel_noise)
    np.testing.assert_array_equal(src.coords()['z'], inst.coords['z'])
