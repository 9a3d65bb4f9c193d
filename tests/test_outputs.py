"""Output types at the Workflow boundary (CPU; no engine calls).

The reference's workflows return ``scipp.DataArray`` values with window time
coords made by ``Timestamp.to_scipp()`` -- 0-D int64 scalars with unit 'ns'
(SRC/core/timestamp.py:216-220; SRC/workflows/stream_processor_workflow.py:
229-238) -- which ``Job._add_time_coords`` (SRC/core/job.py:212-262) and
``scipp_to_da00`` (SRC/kafka/scipp_da00_compat.py:22-116) consume unchanged.
scipp is not importable in this image, so the conversion is checked against a
recording stand-in module.
"""

import sys
import types

import numpy as np
import pytest

from esslivedata_amd import dataarray as dam
from esslivedata_amd import da00
from esslivedata_amd.dataarray import DataArray, Variable
from esslivedata_amd.preprocessors import Timestamp


class _FakeVar:
    def __init__(self, kind, dims, value, unit, dtype):
        self.kind, self.dims, self.value, self.unit, self.dtype = kind, dims, value, unit, dtype


class _FakeDataArray:
    def __init__(self, data, coords=None):
        self.data, self.coords = data, dict(coords or {})

    def assign_coords(self, **coords):
        return _FakeDataArray(self.data, {**self.coords, **coords})


@pytest.fixture
def fake_scipp(monkeypatch):
    mod = types.ModuleType('scipp')
    mod.scalar = lambda value, unit=None, dtype=None: _FakeVar('scalar', (), value, unit, dtype)
    mod.array = lambda dims, values, unit=None, dtype=None: _FakeVar('array', tuple(dims), values,
                                                                     unit, dtype)
    mod.DataArray = _FakeDataArray
    monkeypatch.setitem(sys.modules, 'scipp', mod)
    dam.reset_scipp_module()
    yield mod
    dam.reset_scipp_module()


def test_scipp_probe_cached_and_absent_here():
    dam.reset_scipp_module()
    assert dam.scipp_module() is None  # not importable in this image
    assert dam._SCIPP == [None]        # probed once, not per finalize


def test_timestamp_to_scipp_standin_is_int64_ns():
    v = Timestamp.from_ns(1000).to_scipp()
    assert isinstance(v, Variable) and v.dims == () and v.unit == 'ns'
    assert v.value == 1000 and np.asarray(v.values).dtype == np.int64


def test_timestamp_to_scipp_with_scipp(fake_scipp):
    v = Timestamp.from_ns(2000).to_scipp()
    assert v.kind == 'scalar' and v.value == 2000 and v.unit == 'ns' and v.dtype == 'int64'


def test_publish_converts_with_dtypes(fake_scipp):
    st = Timestamp.from_ns(5).to_scipp()
    img = DataArray(np.ones((2, 3), np.float32), ('y', 'x'), 'counts',
                    {'x': Variable(('x',), np.arange(3.0), 'm')})
    tot = DataArray(np.asarray(np.float32(6)), (), 'counts').assign_coords(start_time=st, time=st)
    echo = object()  # a caller's own ROI request passes through
    out = dam.publish({'current': img, 'counts_total': tot, 'roi_rectangle': echo})
    cur = out['current']
    assert isinstance(cur, _FakeDataArray)
    assert cur.data.dims == ('y', 'x') and cur.data.dtype == 'float32' and cur.data.unit == 'counts'
    assert cur.coords['x'].unit == 'm' and cur.coords['x'].dtype == 'float64'
    t = out['counts_total']
    assert t.data.kind == 'scalar' and t.data.dtype == 'float32'
    # the stamped time coords were already scipp scalars (made by to_scipp)
    assert t.coords['start_time'] is st
    assert out['roi_rectangle'] is echo


def test_publish_without_scipp_returns_standins():
    dam.reset_scipp_module()
    d = {'a': DataArray(np.zeros(2), ('x',))}
    assert dam.publish(d) is d


def test_add_time_coords_mirrors_job():
    """job.py:212-262: stamp every DataArray lacking start_time / time; skip
    those that carry either; no bounds -> ValueError."""
    win = DataArray(np.zeros(2), ('x',)).assign_coords(start_time=Timestamp.from_ns(1).to_scipp())
    cum = DataArray(np.zeros(2), ('x',))
    out = dam.add_time_coords({'current': win, 'cumulative': cum, 'n': 3},
                              Timestamp.from_ns(10), Timestamp.from_ns(20))
    assert 'time' not in out['current'].coords  # skipped: it has start_time
    assert out['cumulative'].coords['start_time'].value == 10
    assert out['cumulative'].coords['time'].value == 20
    assert np.asarray(out['cumulative'].coords['time'].values).dtype == np.int64
    assert out['n'] == 3
    with pytest.raises(ValueError, match='no time bounds'):
        dam.add_time_coords({}, None, Timestamp.from_ns(1))


def test_int64_ns_coords_through_da00():
    """An int64 'ns' scalar coord is written as int64 with unit 'ns' and read
    back unchanged (the dashboard's _extract_time_bounds_as_scalars sees the
    same dtype on window and Job-stamped outputs)."""
    st, tt = Timestamp.from_ns(1000).to_scipp(), Timestamp.from_ns(2000).to_scipp()
    da = DataArray(np.arange(3.0), ('t',), 'counts').assign_coords(start_time=st, time=tt)
    variables = da00.dataarray_to_da00(da)
    by = {v.name: v for v in variables}
    assert by['start_time'].unit == 'ns' and by['start_time'].data.dtype == np.int64
    back = da00.da00_to_dataarray(da00.deserialise_da00(da00.serialise_da00('s', 0, variables))[2])
    assert back.coords['time'].value == 2000 and back.coords['time'].unit == 'ns'
    assert np.asarray(back.coords['time'].values).dtype == np.int64


def test_add_time_coords_stamps_published_scipp_arrays(fake_scipp):
    """with scipp present, finalize hands over scipp.DataArray
    values; the Job's stamp must reach them too (job.py:251-259 stamps every
    DataArray), with int64 'ns' scalars."""
    out = dam.publish({'cumulative': DataArray(np.zeros(2), ('x',)), 'n': 3})
    assert isinstance(out['cumulative'], _FakeDataArray)
    st = dam.add_time_coords(out, Timestamp.from_ns(10), Timestamp.from_ns(20))
    c = st['cumulative'].coords
    assert c['start_time'].value == 10 and c['time'].value == 20
    assert c['time'].unit == 'ns' and c['time'].dtype == 'int64'
    assert st['n'] == 3


@pytest.mark.parametrize('bad', [np.array(['a', 'b']), np.array([object(), 1], dtype=object),
                                 np.array([1, 2], dtype=np.uint64)])
def test_scipp_conversion_refuses_dtypes_without_a_scipp_match(fake_scipp, bad):
    with pytest.raises(TypeError, match='no scipp dtype'):
        DataArray(bad, ('x',)).to_scipp()
