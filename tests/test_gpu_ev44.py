"""GPU: ev44 payloads staged by lde_stage_ev44 bin exactly like the decoded
arrays (and like the oracle); rejected payloads stage nothing.

Reference chain: KafkaToEv44Adapter -> Ev44ToDetectorEventsAdapter ->
ToNXevent_data.add (SRC/kafka/message_adapter.py:192-204, 412-437;
SRC/preprocessors/to_nxevent_data.py:16-19, 57-69, 127-153) and
KafkaToMonitorEventsAdapter (message_adapter.py:380-409).
"""

import numpy as np
import pytest

from oracle import scipp_semantics as ora

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _gpu(engine_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def _split_messages(n, cuts):
    bounds = [0, *cuts, n]
    return list(zip(bounds[:-1], bounds[1:]))


def test_detector_ev44_staging_matches_array_staging_and_oracle():
    from esslivedata_amd import ev44, projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.dummy_panel()
    view = projection.logical_lut(inst.detector_number)
    edges = inst.edges.edges_ns()
    pid, toa = synthetic.fake_detector_events(200_003, 1, 16384 + 50, seed=1234)
    msgs = _split_messages(len(pid), [1, 70_001, 70_002, 150_000])

    def engine():
        return BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                             n_screen=view.n_screen)

    a, b = engine(), engine()
    t0 = 1_767_225_600 * 10**9
    for k, (lo, hi) in enumerate(msgs):
        a.stage(pid[lo:hi], toa[lo:hi])
        payload = ev44.serialise_ev44('panel_0', k, [t0 + k], 0, toa[lo:hi], pid[lo:hi])
        assert b.stage_ev44(payload, 99).to_ns() == t0 + k
        # rejected payloads between good ones stage nothing
        with pytest.raises(ValueError):
            b.stage_ev44(payload[:12])
        with pytest.raises(ValueError, match='same length'):
            b.stage_ev44(ev44.serialise_ev44('panel_0', 0, [t0], 0, toa[lo:hi], pid[lo:hi][:-1]))
        with pytest.raises(NotImplementedError):
            b.stage_ev44(ev44.serialise_ev44('panel_0', 0, [t0, t0 + 1], [0, 1], toa[lo:hi],
                                             pid[lo:hi]))
    # an empty message with an empty reference_time: Kafka-timestamp fallback
    assert b.stage_ev44(ev44.serialise_ev44('panel_0', 0, [], 0, [], []), 1234).to_ns() == 1234 * 10**6
    a.accumulate(0)
    b.accumulate(0)
    got = b.read_histogram()
    np.testing.assert_array_equal(got, a.read_histogram())
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=np.arange(16384)[None, :],
        screen_shape=(128, 128),
        toa_edges_ns=edges,
    )
    np.testing.assert_array_equal(got, o.batch_histogram(pid, toa, 0).reshape(got.shape))


def test_monitor_ev44_staging_ignores_pixel_id():
    from esslivedata_amd import ev44, synthetic
    from esslivedata_amd.engine import BinningEngine

    edges = np.linspace(0.0, 71_000_000.0, 101)
    _, toa = synthetic.uniform_events(50_000, 1, 2, seed=2)
    a = BinningEngine.monitor(edges)
    b = BinningEngine.monitor(edges)
    a.stage(None, toa)
    # mismatched vectors are accepted on the plain monitor path
    # (tests/kafka/adapter_robustness_test.py:84-97), multi-pulse too (no check)
    payload = ev44.serialise_ev44('monitor1', 0, [5, 6], [0, 1], toa, np.zeros(3, dtype=np.int32))
    assert b.stage_ev44(payload, single_pulse=False).to_ns() == 6
    a.accumulate(0)
    b.accumulate(0)
    np.testing.assert_array_equal(a.read_histogram(), b.read_histogram())
    np.testing.assert_array_equal(b.read_histogram().ravel(), np.histogram(toa, edges)[0])


def test_threaded_host_staging_large_messages():
    """lde_stage splits large messages over worker threads (each chunk's H2D
    queued by the thread that copied it): detector and monitor handles, ragged
    chunk tails, a message that starts mid-ring."""
    from esslivedata_amd import ev44, projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.dummy_panel()
    view = projection.logical_lut(inst.detector_number)
    edges = inst.edges.edges_ns()
    pid, toa = synthetic.fake_detector_events(3_333_337, 1, 16384 + 50, seed=9)
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen)
    eng.stage(pid[:7], toa[:7])
    eng.stage_ev44(ev44.serialise_ev44('panel_0', 0, [1], 0, toa[7:], pid[7:]))
    eng.accumulate(0)
    o = ora.OracleDetectorView(detector_number=inst.detector_number,
                               pixel_screen=np.arange(16384)[None, :], screen_shape=(128, 128),
                               toa_edges_ns=edges)
    got = eng.read_histogram()
    np.testing.assert_array_equal(got, o.batch_histogram(pid, toa, 0).reshape(got.shape))
    mon = BinningEngine.monitor(np.linspace(0.0, 80_000_000.5, 101))
    mon.stage(None, toa)
    mon.accumulate(0)
    np.testing.assert_array_equal(mon.read_histogram().ravel(),
                                  np.histogram(toa, np.linspace(0.0, 80_000_000.5, 101))[0])
