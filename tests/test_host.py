"""Host-side logic (CPU only): LUT construction, edges, preprocessing contract."""

import numpy as np
import pytest

from oracle import scipp_semantics as ora


def test_geometric_lut_matches_oracle_all_replicas():
    from esslivedata_amd import projection

    rng = np.random.default_rng(0)
    p, r = 5000, 3
    dn = np.arange(1000, 1000 + 2 * p, 2)  # non-contiguous ids
    coords = {'x': rng.normal(0, 1, (r, p)), 'y': rng.normal(0, 2, (r, p))}
    coords['x'][1, 7] = np.nan
    res = {'y': 13, 'x': 17}
    view = projection.geometric_lut(dn, coords, res, flip_x=True)
    oc = {'x': -coords['x'], 'y': coords['y']}
    edges = {d: ora.screen_edges(oc[d], n) for d, n in res.items()}
    assert view.screen_dims == ('y', 'x') and view.screen_shape == (13, 17)
    for k in range(r):
        exp = ora.geometric_screen_index(oc, edges, k)
        got = view.lut[k, dn - view.pid_offset]
        np.testing.assert_array_equal(got, exp)
    # gaps between ids are dropped
    assert (view.lut[:, 1::2] == -1).all()
    assert view.lut[1, dn[7] - view.pid_offset] == -1  # NaN coordinate
    # pixel weights: mean pixels per screen bin over replicas
    w = np.zeros(13 * 17)
    for k in range(r):
        s = view.lut[k][view.lut[k] >= 0]
        w += np.bincount(s, minlength=13 * 17)
    np.testing.assert_allclose(view.pixel_weights.ravel(), (w / r).astype(np.float32))


def test_logical_lut_identity_and_bifrost_fold():
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dummy_panel()
    v = projection.logical_lut(inst.detector_number, dims=('y', 'x'))
    assert v.screen_shape == (128, 128) and v.screen_dims == ('y', 'x')
    np.testing.assert_array_equal(v.lut[0], np.arange(128 * 128))
    b = synthetic.bifrost_unified()
    vb = projection.logical_lut(b.detector_number, transform=synthetic.bifrost_transform)
    assert vb.screen_shape == (15, 900)
    exp, shape = ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)
    np.testing.assert_array_equal(vb.lut[0], exp)


def test_logical_lut_with_reduction_and_slice():
    from esslivedata_amd import projection

    dn = np.arange(1, 25).reshape(4, 6)
    v = projection.logical_lut(dn, transform=lambda a: a.T[1:], reduction_axes=(1,))
    exp, shape = ora.logical_screen_index((4, 6), lambda a: a.T[1:], reduction_axes=(1,))
    assert v.screen_shape == shape
    np.testing.assert_array_equal(v.lut[0], exp)
    np.testing.assert_array_equal(v.pixel_weights, [4, 4, 4, 4, 4])


def test_pid_table_rejects_duplicates_and_huge_ranges():
    from esslivedata_amd import projection

    with pytest.raises(ValueError, match='duplicate'):
        projection.pid_pixel_table(np.array([1, 2, 2]))
    with pytest.raises(ValueError):
        projection.pid_pixel_table(np.array([0, 2**29]))


def test_toa_edges_model():
    from esslivedata_amd.edges import ESS_PULSE_PERIOD_MS, TOAEdges, convert_time, label_slice

    assert ESS_PULSE_PERIOD_MS == 71.43
    e = TOAEdges()
    np.testing.assert_array_equal(e.edges_ns(), np.linspace(0, 71.43, 101) * 1e6)
    np.testing.assert_array_equal(
        TOAEdges(start=0.5, scale='log').edges_ns(), np.geomspace(0.5, 71.43, 101) * 1e6
    )
    with pytest.raises(ValueError):
        TOAEdges(start=2.0, stop=1.0)
    with pytest.raises(ValueError):
        TOAEdges(start=0.0, scale='log')
    with pytest.raises(ValueError):
        TOAEdges(num_bins=0)
    edges = np.array([0.0, 2.0, 4.0, 6.0, 8.0, 10.0])
    for lo, hi in [(2, 8), (1, 7), (-3, 30), (4, 4), (9.9, 10)]:
        assert label_slice(edges, lo, hi) == ora.label_slice(edges, lo, hi)
    np.testing.assert_array_equal(convert_time(np.array([1.5]), 'ms', 'ns'), [1.5e6])


def test_event_staging_contract():
    """Error conventions of ToNXevent_data (to_nxevent_data.py:140-204)."""
    from esslivedata_amd.preprocessors import (
        DetectorEvents,
        EventStaging,
        MonitorEvents,
        Timestamp,
    )

    acc = EventStaging()
    with pytest.raises(ValueError, match='No data'):
        acc.get()
    with pytest.raises(ValueError, match="unit 'ns'"):
        acc.add(Timestamp.from_ns(0), MonitorEvents([1, 2], unit='us'))
    acc.add(Timestamp.from_ns(1), DetectorEvents(pixel_id=[1, 2], time_of_arrival=[5, 6], unit='ns'))
    with pytest.raises(ValueError, match='Inconsistent'):
        acc.add(Timestamp.from_ns(2), MonitorEvents([1], unit='ns'))
    acc.add(Timestamp.from_ns(3), DetectorEvents(pixel_id=np.array([3]), time_of_arrival=np.array([7]), unit='ns'))
    out = acc.get()
    assert out.n_messages == 2 and out.n_events == 3 and out.event_time_zero == [1, 3]
    assert all(a.dtype == np.int32 for a in out.time_of_arrival + out.pixel_id)
    with pytest.raises(RuntimeError, match='not been released'):
        acc.get()
    acc.release_buffers()
    out = acc.get()  # after release: empty batch, same stream type
    assert out.n_events == 0
    with pytest.raises(ValueError, match='same length'):
        DetectorEvents(pixel_id=[1, 2], time_of_arrival=[1], unit='ns')


def test_multi_pulse_ev44_rejected():
    from esslivedata_amd.preprocessors import DetectorEvents

    class Ev44:
        reference_time_index = np.array([0, 5])
        reference_time = np.array([1, 2])
        pixel_id = np.array([1])
        time_of_flight = np.array([1])

    with pytest.raises(NotImplementedError):
        DetectorEvents.from_ev44(Ev44())


def test_preprocessor_factory_skips_unconfigured():
    from esslivedata_amd.preprocessors import (
        EventStaging,
        GpuPreprocessorFactory,
        StreamId,
        StreamKind,
    )

    f = GpuPreprocessorFactory(detector_numbers={'panel_0': np.arange(1, 5)})
    assert isinstance(f.make_preprocessor(StreamId(StreamKind.DETECTOR_EVENTS, 'panel_0')), EventStaging)
    assert f.make_preprocessor(StreamId(StreamKind.DETECTOR_EVENTS, 'other')) is None
    assert isinstance(f.make_preprocessor(StreamId(StreamKind.MONITOR_EVENTS, 'm1')), EventStaging)


def test_product_package_never_imports_oracle():
    """The shipped package must not route through the CPU oracle."""
    from pathlib import Path

    pkg = Path(__file__).resolve().parents[1] / 'esslivedata_amd'
    for f in pkg.rglob('*.py'):
        text = f.read_text()
        assert 'import oracle' not in text and 'from oracle' not in text, f


def test_wide_pixel_ids_are_dropped_not_wrapped():
    """An int64 id of 2**32 + 5 is an unknown id (dropped, group_by_pixel.py:
    46-54), not pixel 5; a TOA beyond int32 is refused (the ev44 field is
    int32).  Conversion only; nothing runs on a device."""
    from esslivedata_amd.engine import _as_i32

    pid = np.array([5, 2**32 + 5, -(2**31) - 1, 7], dtype=np.int64)
    out = _as_i32(pid, 'pixel_id', unknown_id=0)
    np.testing.assert_array_equal(out, [5, 0, 0, 7])
    assert out.dtype == np.int32
    np.testing.assert_array_equal(_as_i32(np.array([3, 2**40], dtype=np.uint64), 'pixel_id', -1), [3, -1])
    np.testing.assert_array_equal(_as_i32(np.array([1, 2], dtype=np.int64), 'toa'), [1, 2])
    with pytest.raises(ValueError):
        _as_i32(np.array([2**31], dtype=np.int64), 'time_of_arrival')
    with pytest.raises(TypeError):
        _as_i32(np.array([1.0]), 'pixel_id', 0)
    # the staging accumulator keeps wide arrays unconverted for the engine
    from esslivedata_amd.preprocessors import DetectorEvents, EventStaging, Timestamp

    st = EventStaging()
    st.add(Timestamp.from_ns(0), DetectorEvents(pixel_id=pid, time_of_arrival=np.arange(4),
                                                unit='ns'))
    assert st.get().pixel_id[0].dtype == np.int64


def test_bench_launcher_refuses_more_ranks_than_gpus(monkeypatch):
    """``bench.py --gpus N`` over RCCL refuses N beyond the visible GPUs
    (without initialising HIP in the launching process)."""
    import subprocess

    import bench

    class A:
        gpus = 4

    monkeypatch.setenv('LDE_BENCH_BACKEND', 'nccl')
    monkeypatch.setattr(subprocess, 'run', lambda *a, **k: pytest.fail('must not launch'))
    assert bench.launch_ranks(A()) == 2


def test_bench_launcher_command(monkeypatch):
    """The launcher starts torch.distributed.run with N ranks on 127.0.0.1 and
    passes its own arguments through."""
    import subprocess
    import sys

    import bench

    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env=None, **k):
        seen['cmd'], seen['env'] = cmd, env
        return R()

    class A:
        gpus = 3

    monkeypatch.setenv('LDE_BENCH_BACKEND', 'gloo')
    monkeypatch.setattr(subprocess, 'run', fake_run)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '3', '--steps', '2'])
    assert bench.launch_ranks(A()) == 0
    cmd = seen['cmd']
    assert cmd[1:3] == ['-m', 'torch.distributed.run']
    assert '--nproc-per-node=3' in cmd and '--master-addr=127.0.0.1' in cmd
    assert cmd[-4:] == ['--gpus', '3', '--steps', '2']
