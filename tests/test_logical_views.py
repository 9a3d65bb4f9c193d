"""Logical views by dim name (row A8): the LogicalIndex stand-in for the
reference's scipp transforms, the DREAM / MAGIC views against the oracle's
closed-form index, and the reference's own logical-projection KATs
(tests/golden/reference_kats.json) through the oracle.  CPU only."""

import json
from pathlib import Path

import numpy as np
import pytest

from esslivedata_amd import projection, synthetic
from esslivedata_amd.logical import LogicalIndex, detector_index
from oracle import scipp_semantics as ora

REF = {k['name']: k for k in json.loads(
    (Path(__file__).resolve().parent / 'golden' / 'reference_kats.json').read_text())}

# closed-form (oracle) description of each DREAM view: output axes, fixed dims
DREAM_SPEC = {
    'mantle_front_layer': ([('module', 'segment', 'counter'), ('strip',)], {'wire': 0}),
    'wire_view': ([('wire',), ('module', 'segment', 'counter')], {}),
    'strip_view': ([('strip',)], {}),
}
MAGIC_SPEC = {
    'wire_view': [('wire',), ('segment',)],
    'strip_view': [('strip',)],
}


def test_logical_index_follows_scipp_structure_rules():
    x = detector_index(np.arange(24))
    assert x.dim == 'detector_number'
    f = x.fold(dim=x.dim, sizes={'a': 2, 'b': -1, 'c': 4})
    assert f.sizes == {'a': 2, 'b': 3, 'c': 4}
    np.testing.assert_array_equal(f.values, np.arange(24).reshape(2, 3, 4))
    t = f.transpose(('c', 'a', 'b'))
    np.testing.assert_array_equal(t.values, np.arange(24).reshape(2, 3, 4).transpose(2, 0, 1))
    fl = t.flatten(('a', 'b'), to='ab')
    assert fl.dims == ('c', 'ab')
    np.testing.assert_array_equal(fl.values, np.arange(24).reshape(2, 3, 4).transpose(2, 0, 1).reshape(4, 6))
    s = f['b', 1]
    assert s.dims == ('a', 'c')
    np.testing.assert_array_equal(s.values, np.arange(24).reshape(2, 3, 4)[:, 1])
    assert f['b', 1:3].sizes == {'a': 2, 'b': 2, 'c': 4}
    with pytest.raises(ValueError):
        f.flatten(('a', 'c'), to='ac')  # not adjacent: scipp refuses
    with pytest.raises(ValueError):
        x.fold(dim=x.dim, sizes={'a': 5, 'b': -1})
    with pytest.raises(ValueError):
        _ = f.dim  # multi-dim
    with pytest.raises(IndexError):
        f['a', 2]
    assert isinstance(x.to(dtype='float32'), LogicalIndex)  # value-only ops are no-ops


@pytest.mark.parametrize('name', list(DREAM_SPEC))
def test_dream_views_match_the_closed_form_index(name):
    cfg = synthetic.dream_logical_views()[name]
    inst_dn = np.arange(229377, 720897, dtype=np.int32)
    v = projection.logical_lut(inst_dn, transform=lambda a: cfg.transform(a, 'mantle_detector'),
                               reduction_dim=cfg.reduction_dim)
    sizes = synthetic.DREAM_BANK_SIZES['mantle_detector']
    assert int(np.prod(list(sizes.values()))) == inst_dn.size == 491520
    exp, shape = ora.folded_view_index(sizes, *DREAM_SPEC[name])
    assert v.screen_shape == shape
    np.testing.assert_array_equal(v.lut[0], exp)
    # pixel weights: detector pixels merged into each output pixel
    # (LogicalProjector.compute_weights, projectors.py:272-303)
    w = np.bincount(exp[exp >= 0], minlength=int(np.prod(shape))).reshape(shape)
    np.testing.assert_array_equal(v.pixel_weights, w.astype(np.float32))


def test_dream_view_dims_and_sizes():
    views = synthetic.dream_logical_views()
    dn = np.arange(229377, 720897, dtype=np.int32)
    got = {}
    for name, cfg in views.items():
        v = projection.logical_lut(dn, transform=lambda a: cfg.transform(a, 'mantle_detector'),
                                   reduction_dim=cfg.reduction_dim)
        got[name] = dict(zip(v.screen_dims, v.screen_shape))
    # dream/views.py:13-85 docstrings: (mod/seg/cntr, strip) for the front
    # layer, (wire, mod/seg/cntr) after reducing strip, (strip,) after other
    assert got['mantle_front_layer'] == {'mod/seg/cntr': 60, 'strip': 256}
    assert got['wire_view'] == {'wire': 32, 'mod/seg/cntr': 60}
    assert got['strip_view'] == {'strip': 256}
    assert not views['wire_view'].roi_support and not views['strip_view'].roi_support


def test_magic_views_conserve_counts_kat():
    kat = REF['magic_views_conserve_counts']
    views = synthetic.magic_logical_views()
    for bank, exp in kat['banks'].items():
        inst = synthetic.magic_bank(bank)
        assert inst.detector_number.size == exp['pixel_count']
        counts = np.random.default_rng(seed=1).integers(0, 5, size=exp['pixel_count'])
        for vname in ('wire_view', 'strip_view'):
            cfg = views[vname]
            assert cfg.reduction_dim == kat[vname]['reduction_dim']
            v = projection.logical_lut(inst.detector_number,
                                       transform=lambda a: cfg.transform(a, bank),
                                       reduction_dim=cfg.reduction_dim)
            assert list(v.screen_dims) == kat[vname]['expected_dims']
            for d in v.screen_dims:
                assert v.screen_shape[v.screen_dims.index(d)] == exp[d]
            reduced = np.bincount(v.lut[0], weights=counts, minlength=v.n_screen)
            assert reduced.sum() == counts.sum()
            o, shape = ora.folded_view_index(synthetic.MAGIC_BANK_SIZES[bank], MAGIC_SPEC[vname])
            np.testing.assert_array_equal(v.lut[0], o)


def _fold_view(kat, reduction_dim):
    sizes = kat['fold_sizes']
    dn = np.arange(1, int(np.prod(list(sizes.values()))) + 1, dtype=np.int32)
    return projection.logical_lut(dn, transform=lambda a: a.fold(dim='detector_number', sizes=sizes),
                                  reduction_dim=reduction_dim), dn


def test_logical_screen_metadata_kat():
    kat = REF['logical_screen_metadata']
    for case in kat['cases']:
        v, _ = _fold_view(kat, case['reduction_dim'])
        assert dict(zip(v.screen_dims, v.screen_shape)) == case['expected_sizes']


def test_logical_reduction_conserves_events_kat():
    kat = REF['logical_reduction_concatenates_events']
    for case in kat['cases']:
        v, dn = _fold_view(kat, case['reduction_dim'])
        assert list(v.screen_dims) == case['expected_dims']
        assert dict(zip(v.screen_dims, v.screen_shape)) == case['expected_sizes']
        event_id = np.repeat(dn, kat['n_events_per_pixel'])
        toa = np.random.default_rng(42).uniform(0, 71_000_000, event_id.size).astype(np.int32)
        edges = ora.to_ns(ora.make_edges(0.0, ora.ESS_PULSE_PERIOD_MS, 100), 'ms')
        h = ora.detector_histogram(v.lut[0], v.n_screen, ora.pixel_index(event_id, dn), toa, edges)
        assert h.sum() == case['expected_events']


def test_reduction_dim_must_name_a_transformed_dim():
    dn = np.arange(1, 17, dtype=np.int32)
    with pytest.raises(ValueError):
        projection.logical_lut(dn, transform=lambda a: a.fold(dim='detector_number',
                                                               sizes={'y': 4, 'x': 4}),
                               reduction_dim='z')
    with pytest.raises(ValueError):  # names need a named result
        projection.logical_lut(dn, transform=lambda a: a.reshape(4, 4), reduction_dim='y')


def test_factory_accepts_reduction_dim_by_name():
    from esslivedata_amd.workflows import GpuDetectorViewFactory, LogicalViewConfig

    cfg = LogicalViewConfig(transform=lambda da, s: da.fold(dim=da.dim, sizes={'y': 4, 'x': 4}),
                            reduction_dim='y')
    fac = GpuDetectorViewFactory(detector_numbers={'det': np.arange(1, 17, dtype=np.int32)},
                                 view_config=cfg)
    v = fac.make_view('det')
    assert v.screen_dims == ('x',) and v.screen_shape == (4,)
    np.testing.assert_array_equal(v.pixel_weights, np.full(4, 4, dtype=np.float32))
