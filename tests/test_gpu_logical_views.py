"""DREAM logical views on the GPU at headline size (row A8).

The mantle's ``mantle_front_layer`` (slice ``['wire', 0]``), ``wire_view``
(reduce ``strip``) and ``strip_view`` (reduce ``other``: every event lands in
one of 256 screens, the path's hottest shape) are built through
``GpuDetectorViewFactory(LogicalViewConfig(...))`` from the restated
transforms (dream/views.py:13-85, dream/specs.py:151-180) and bin 1.4e8 Zipf
events as 14 x 1e7 device messages per step over two finalizes, for AUTO and
every forced strategy.  The current and cumulative histograms, images and
totals are compared bit-exactly with ``oracle/binning_ref.c`` fed the
oracle's closed-form view index (``folded_view_index``, which derives the
pixel -> output map without applying any transform).  The reference's own
logical-projection KATs (providers_test.py:208-348) run through the same
factory.
"""

import json
import os
from pathlib import Path

import numpy as np
import pytest

from oracle import c_oracle
from oracle import scipp_semantics as ora

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

REF = {k['name']: k for k in json.loads(
    (Path(__file__).resolve().parent / 'golden' / 'reference_kats.json').read_text())}

N_PULSE = 10_000_000
PULSES = 14
SOURCE = 'mantle_detector'
DREAM_SPEC = {
    'mantle_front_layer': ([('module', 'segment', 'counter'), ('strip',)], {'wire': 0}),
    'wire_view': ([('wire',), ('module', 'segment', 'counter')], {}),
    'strip_view': ([('strip',)], {}),
}
STRATEGIES = ['auto', 'atomic', 'partition', 'paged', 'split', 'pixel']


@pytest.fixture(scope='module', autouse=True)
def _gpu(engine_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def _t(ns):
    from esslivedata_amd.preprocessors import Timestamp

    return Timestamp.from_ns(ns)


def _threads() -> int:
    return int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0))


@pytest.fixture(scope='module')
def dream_steps():
    """Two steps of 1.4e8 DREAM events (bench generator, seeds 7 and 8):
    device messages + host copies."""
    import torch

    from esslivedata_amd import synthetic

    dev = torch.device('cuda', 0)
    inst = synthetic.dream_mantle(n_replicas=1)
    steps = []
    for seed in (7, 8):
        pid, toa = synthetic.torch_dream_events(N_PULSE * PULSES, inst, seed, dev)
        msgs = [(pid[p * N_PULSE:(p + 1) * N_PULSE], toa[p * N_PULSE:(p + 1) * N_PULSE])
                for p in range(PULSES)]
        steps.append((msgs, pid.cpu().numpy(), toa.cpu().numpy()))
    torch.cuda.synchronize()
    return inst, steps


_ORACLE: dict = {}


def _oracle(view_name, inst, steps):
    """Per step: (current, cumulative) (S, T) uint64 histograms."""
    if view_name not in _ORACLE:
        from esslivedata_amd import synthetic

        lut, shape = ora.folded_view_index(synthetic.DREAM_BANK_SIZES[SOURCE],
                                           *DREAM_SPEC[view_name])
        edges = inst.edges.edges_ns()
        S, T = int(np.prod(shape)), len(edges) - 1
        o = c_oracle.CDetectorView(inst.detector_number, lut[None, :], S, edges,
                                   threads=_threads())
        prev = np.zeros(S * T, dtype=np.uint64)
        out = []
        for _, hp, ht in steps:
            cum = o.accumulate(hp, ht, 0).copy()
            out.append(((cum - prev).reshape(S, T), cum.reshape(S, T)))
            prev = cum
        _ORACLE[view_name] = (shape, out)
    return _ORACLE[view_name]


@pytest.mark.parametrize('strategy', STRATEGIES)
@pytest.mark.parametrize('view_name', list(DREAM_SPEC))
def test_dream_logical_view_headline_bit_exact(dream_steps, view_name, strategy):
    import time

    import torch

    from esslivedata_amd import synthetic
    from esslivedata_amd.preprocessors import StagedEvents
    from esslivedata_amd.workflows import DetectorViewParams, GpuDetectorViewFactory

    inst, steps = dream_steps
    shape, expected = _oracle(view_name, inst, steps)
    fac = GpuDetectorViewFactory(detector_numbers={SOURCE: inst.detector_number},
                                 view_config=synthetic.dream_logical_views()[view_name],
                                 strategy=strategy)
    wf = fac.make_workflow(SOURCE, DetectorViewParams(toa_edges=inst.edges))
    assert wf.view.screen_shape == shape
    times = []
    for k, ((msgs, _, _), (cur, cum)) in enumerate(zip(steps, expected)):
        staged = StagedEvents(time_of_arrival=[m[1] for m in msgs],
                              pixel_id=[m[0] for m in msgs], event_time_zero=[k] * len(msgs))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wf.accumulate({SOURCE: staged}, start_time=_t(k), end_time=_t(k + 1))
        hist_cur = wf.read_histogram('current').values
        times.append(time.perf_counter() - t0)
        out = wf.finalize()
        hist_cum = wf.read_histogram('cumulative').values
        np.testing.assert_array_equal(hist_cur.reshape(cur.shape), cur.astype(np.float64))
        np.testing.assert_array_equal(hist_cum.reshape(cum.shape), cum.astype(np.float64))
        np.testing.assert_array_equal(out['current'].values, cur.sum(1).reshape(shape).astype(np.float64))
        np.testing.assert_array_equal(out['cumulative'].values, cum.sum(1).reshape(shape).astype(np.float64))
        assert float(out['counts_total'].values) == float(cur.sum())
        assert float(out['counts_total_cumulative'].values) == float(cum.sum())
        assert out['current'].dims == wf.view.screen_dims
    info = wf.engine.info()
    if strategy != 'auto':
        # forced strategies may fall back (SPLIT -> WIDE / PAGED without a
        # sieve encoding, tiled strategies -> ATOMIC without tiles), never
        # silently to something else
        assert info['last_strategy'] in (strategy, 'wide', 'paged', 'atomic')
    print(f'\n[{view_name} {strategy}] last_strategy={info["last_strategy"]} '
          f'accumulate+read {1e3 * min(times):.2f} ms')
    if view_name == 'mantle_front_layer':
        assert expected[0][0].sum() < 0.1 * N_PULSE * PULSES  # wire 0 only: most events dropped
    else:
        assert expected[0][0].sum() > 0.9 * N_PULSE * PULSES


def _fold(sizes):
    return lambda da, source: da.fold(dim=da.dim, sizes=sizes)


def _factory(kat, reduction_dim, edges=None):
    from esslivedata_amd.edges import TOAEdges
    from esslivedata_amd.workflows import DetectorViewParams, GpuDetectorViewFactory, LogicalViewConfig

    sizes = kat['fold_sizes']
    dn = np.arange(1, int(np.prod(list(sizes.values()))) + 1, dtype=np.int32)
    fac = GpuDetectorViewFactory(detector_numbers={'det': dn},
                                 view_config=LogicalViewConfig(transform=_fold(sizes),
                                                               reduction_dim=reduction_dim))
    params = DetectorViewParams()
    if edges is not None:
        params = DetectorViewParams(toa_edges=TOAEdges(start=edges[0], stop=edges[-1],
                                                       num_bins=len(edges) - 1, unit='ns'))
    return fac.make_workflow('det', params), dn


def test_logical_reduction_kats_through_factory():
    """providers_test.py:249-278: events conserved under reduction over one
    and over both dims (0-D result)."""
    kat = REF['logical_reduction_concatenates_events']
    for case in kat['cases']:
        wf, dn = _factory(kat, case['reduction_dim'])
        pid = np.repeat(dn, kat['n_events_per_pixel'])
        toa = np.random.default_rng(42).uniform(0, 71_000_000, pid.size).astype(np.int32)
        wf.accumulate({'det': (pid, toa)}, start_time=_t(0), end_time=_t(1))
        out = wf.finalize()
        assert list(out['current'].dims) == case['expected_dims']
        assert dict(zip(out['current'].dims, out['current'].values.shape)) == case['expected_sizes']
        assert float(out['counts_total'].values) == case['expected_events']
        assert float(np.sum(out['current'].values)) == case['expected_events']


def test_detector_image_and_counts_total_kats_through_factory():
    """providers_test.py:284-305 (image = 10 per pixel) and :336-348
    (counts_total = 160, current and cumulative) as events: one event per
    (pixel, bin) at the bin centre."""
    kat = REF['detector_image_sums_spectral_dim']
    edges = np.array(kat['edges_ns'])
    wf, dn = _factory(kat, None, edges)
    centres = (0.5 * (edges[1:] + edges[:-1])).astype(np.int32)
    pid = np.repeat(dn, len(centres))
    toa = np.tile(centres, len(dn))
    wf.accumulate({'det': (pid, toa)}, start_time=_t(0), end_time=_t(1))
    out = wf.finalize()
    np.testing.assert_array_equal(out['current'].values, np.full((4, 4), kat['expected_image']))
    tot = REF['counts_total_ones']['expected']
    assert float(out['counts_total'].values) == tot
    assert float(out['counts_total_cumulative'].values) == tot


def test_screen_metadata_kat_through_factory():
    kat = REF['logical_screen_metadata']
    for case in kat['cases']:
        wf, _ = _factory(kat, case['reduction_dim'])
        assert dict(zip(wf.view.screen_dims, wf.view.screen_shape)) == case['expected_sizes']
