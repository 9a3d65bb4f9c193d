"""ev44 decode + adapters on CPU (no compute call; the decoder is host code).

Mirrors the reference's adapter tests:
* tests/kafka/adapter_robustness_test.py:69-167 (containment of the
  hostile-wire corpus, mismatched vectors on the monitor path, absent vectors,
  far-future timestamps crossing verbatim);
* tests/helpers/hostile_wire.py:52-228 (the corpus itself, rebuilt with our
  writer since ess-streaming-data-types is not installed);
* the adapter timestamp fallback, message_adapter.py:197-201.
The native decoder is also checked against the independent pure-Python
reader in oracle/ev44_reader.py (byte layout: parity unpinned, see there).
"""

from __future__ import annotations

import numpy as np
import pytest

from oracle import ev44_reader

SOURCE = 'monitor1'
TOPIC = 'dummy_beam_monitor'
REALISTIC_EPOCH_NS = 1_767_225_600 * 1_000_000_000
FAR_FUTURE_NS = 7_258_118_400 * 1_000_000_000


@pytest.fixture(scope='module')
def ev(engine_lib):
    from esslivedata_amd import ev44

    return ev44


def _events(ev, source_name, *, reference_time_ns, n_events=10, seed=0):
    # hostile_wire.ev44_events (tests/helpers/hostile_wire.py:52-89)
    rng = np.random.default_rng(seed)
    toa = rng.uniform(0, 70_000_000, n_events).astype(np.int32)
    rt = [] if reference_time_ns is None else [reference_time_ns]
    return ev.serialise_ev44(source_name, 0, rt, 0, toa, np.zeros(n_events, dtype=np.int32))


def _corpus(ev, source_name):
    good = _events(ev, source_name, reference_time_ns=REALISTIC_EPOCH_NS)
    wrong = bytearray(good)
    wrong[4:8] = b'f144'
    return {
        'garbage': bytes(range(256)) * 4,
        'empty': b'',
        'truncated_ev44': good[:12],
        'ev44_without_event_vectors': ev.serialise_ev44(
            source_name, 0, [], 0, [], [],
            omit=('reference_time', 'reference_time_index', 'time_of_flight', 'pixel_id')),
        'wrong_schema_f144': bytes(wrong),
        'unmapped_source': _events(ev, 'not_a_known_source', reference_time_ns=REALISTIC_EPOCH_NS),
    }


def _monitor_adapter(ev):
    lut = {ev.InputStreamKey(topic=TOPIC, source_name=SOURCE): SOURCE}
    return ev.KafkaToMonitorEventsAdapter(lut)


def _msg(ev, payload, timestamp_ms=1234):
    return ev.FakeKafkaMessage(value=payload, topic=TOPIC, timestamp=timestamp_ms, timestamp_type=1)


class _ListSource:
    def __init__(self, messages):
        self._messages = list(messages)

    def get_messages(self):
        messages, self._messages = self._messages, []
        return messages


@pytest.mark.parametrize('n', [0, 1, 7, 1000])
@pytest.mark.parametrize('name', ['panel_0', 'unified_detector', 'détecteur'])
def test_round_trip_matches_inputs_and_oracle_reader(ev, n, name):
    rng = np.random.default_rng(n)
    toa = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    pid = rng.integers(0, 2**31, n).astype(np.int32)
    rt = rng.integers(0, 2**62, 3)
    payload = ev.serialise_ev44(name, 42, rt, [0, 1, 2], toa, pid)
    got = ev.deserialise_ev44(payload)
    ref = ev44_reader.read_ev44(payload)
    assert got.source_name == name == ref['source_name']
    assert got.message_id == 42 == ref['message_id']
    for key, want in [('reference_time', rt), ('reference_time_index', [0, 1, 2]),
                      ('time_of_flight', toa), ('pixel_id', pid)]:
        np.testing.assert_array_equal(getattr(got, key), want)
        np.testing.assert_array_equal(ref[key], want)


def test_decoded_vectors_are_views_into_the_payload(ev):
    payload = np.frombuffer(
        ev.serialise_ev44('x', 0, [5], 0, np.arange(4), np.arange(4)), dtype=np.uint8).copy()
    got = ev.deserialise_ev44(payload)
    assert np.shares_memory(got.time_of_flight, payload)
    assert np.shares_memory(got.pixel_id, payload)


@pytest.mark.parametrize('case', ['garbage', 'empty', 'truncated_ev44', 'wrong_schema_f144'])
def test_malformed_payloads_fail_to_decode(ev, case):
    with pytest.raises(ValueError):
        ev.deserialise_ev44(_corpus(ev, SOURCE)[case])


@pytest.mark.parametrize('case', ['garbage', 'empty', 'truncated_ev44', 'ev44_without_event_vectors',
                                  'wrong_schema_f144', 'unmapped_source'])
def test_malformed_payload_is_contained_and_does_not_affect_next_message(ev, case):
    # adapter_robustness_test.py:69-81
    good = _events(ev, SOURCE, reference_time_ns=REALISTIC_EPOCH_NS)
    source = ev.AdaptingMessageSource(
        source=_ListSource([_msg(ev, _corpus(ev, SOURCE)[case]), _msg(ev, good)]),
        adapter=_monitor_adapter(ev))
    adapted = source.get_messages()
    assert len(adapted) == 1
    assert adapted[0].timestamp.to_ns() == REALISTIC_EPOCH_NS


def test_mismatched_event_vectors_accepted_on_plain_monitor_path(ev):
    # adapter_robustness_test.py:84-97 (hostile_wire.py:115-135)
    payload = ev.serialise_ev44(SOURCE, 0, [REALISTIC_EPOCH_NS], 0, np.arange(10),
                                np.zeros(5, dtype=np.int32))
    adapted = _monitor_adapter(ev).adapt(_msg(ev, payload))
    assert adapted.timestamp.to_ns() == REALISTIC_EPOCH_NS
    assert len(adapted.value.time_of_arrival) == 10
    # the detector path checks the lengths (to_nxevent_data.py:57-62)
    chain = ev.ChainedAdapter(ev.KafkaToEv44Adapter(), ev.Ev44ToDetectorEventsAdapter())
    with pytest.raises(ValueError, match='same length'):
        chain.adapt(_msg(ev, payload))


def test_absent_event_vectors_are_dropped_like_the_reference(ev):
    # adapter_robustness_test.py:100-108 is a strict xfail: the message raises
    payload = _corpus(ev, SOURCE)['ev44_without_event_vectors']
    assert ev44_reader.read_ev44(payload)['reference_time'] is None
    with pytest.raises(ValueError, match='absent'):
        _monitor_adapter(ev).adapt(_msg(ev, payload, timestamp_ms=5678))


@pytest.mark.parametrize('which', ['detector', 'monitor'])
def test_far_future_timestamp_crosses_adapter_boundary_verbatim(ev, which):
    # adapter_robustness_test.py:110-167
    payload = _events(ev, SOURCE, reference_time_ns=FAR_FUTURE_NS)
    adapter = ev.KafkaToEv44Adapter() if which == 'detector' else _monitor_adapter(ev)
    source = ev.AdaptingMessageSource(source=_ListSource([_msg(ev, payload)]), adapter=adapter)
    assert [m.timestamp.to_ns() for m in source.get_messages()] == [FAR_FUTURE_NS]


def test_empty_reference_time_falls_back_to_kafka_timestamp(ev):
    payload = _events(ev, SOURCE, reference_time_ns=None)
    adapted = _monitor_adapter(ev).adapt(_msg(ev, payload, timestamp_ms=5678))
    assert adapted.timestamp.to_ns() == 5678 * 1_000_000
    assert ev44_reader.adapt_timestamp_ns(ev44_reader.read_ev44(payload), 5678) == 5678 * 10**6


def test_detector_chain_single_pulse_and_merge(ev):
    chain = ev.ChainedAdapter(ev.KafkaToEv44Adapter(),
                              ev.Ev44ToDetectorEventsAdapter(merge_detectors=True))
    good = ev.serialise_ev44('bank3', 0, [11], 0, np.arange(4), np.arange(4) + 100)
    out = chain.adapt(_msg(ev, good))
    assert out.stream.name == 'unified_detector'
    np.testing.assert_array_equal(out.value.pixel_id, np.arange(4) + 100)
    multi = ev.serialise_ev44('bank3', 0, [11, 12], [0, 2], np.arange(4), np.arange(4))
    with pytest.raises(NotImplementedError):
        chain.adapt(_msg(ev, multi))
    with pytest.raises(NotImplementedError):
        ev44_reader.require_single_pulse(ev44_reader.read_ev44(multi))


def test_pixellated_monitor_keeps_pixel_id(ev):
    lut = {ev.InputStreamKey(topic=TOPIC, source_name=SOURCE): SOURCE}
    adapter = ev.KafkaToMonitorEventsAdapter(lut, pixellated_sources=frozenset({SOURCE}))
    payload = ev.serialise_ev44(SOURCE, 0, [1], 0, np.arange(3), np.array([7, 8, 9]))
    out = adapter.adapt(_msg(ev, payload))
    np.testing.assert_array_equal(out.value.pixel_id, [7, 8, 9])


def test_fuzzed_payloads_never_read_out_of_bounds(ev):
    """Truncations and byte flips: whenever the native decoder accepts a
    payload, the independent reader accepts it too and agrees field by field;
    every returned vector lies inside the payload."""
    rng = np.random.default_rng(3)
    base = ev.serialise_ev44('panel_0', 9, [123], 0, np.arange(50), np.arange(50) * 3)
    accepted = 0
    for trial in range(3000):
        b = bytearray(base)
        if trial % 3 == 0:
            b = b[: rng.integers(0, len(b))]
        else:
            for _ in range(rng.integers(1, 4)):
                b[rng.integers(0, len(b))] = rng.integers(0, 256)
        payload = bytes(b)
        try:
            raw, view = ev.decode_view(payload)
        except ValueError:
            continue
        accepted += 1
        base_addr = raw.ctypes.data
        for ptr, n, size in [(view.reference_time, view.n_reference_time, 8),
                             (view.time_of_flight, view.n_time_of_flight, 4),
                             (view.pixel_id, view.n_pixel_id, 4),
                             (view.reference_time_index, view.n_reference_time_index, 4),
                             (view.source_name, view.source_name_len, 1)]:
            if ptr:
                assert base_addr <= ptr and ptr + n * size <= base_addr + len(payload)
        try:  # a flipped name byte fails utf-8 decoding in both (ValueError)
            got = ev.deserialise_ev44(payload)
        except UnicodeDecodeError:
            with pytest.raises(UnicodeDecodeError):
                ev44_reader.read_ev44(payload)
            continue
        ref = ev44_reader.read_ev44(payload)
        for key in ('reference_time', 'reference_time_index', 'time_of_flight', 'pixel_id'):
            if getattr(got, key) is None:
                assert ref[key] is None
            else:
                np.testing.assert_array_equal(getattr(got, key), ref[key])
    assert accepted > 100
