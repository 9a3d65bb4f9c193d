"""GPU parity: HIP engine (through the C ABI) vs the CPU oracle, bit-exact.

Counts are integers, so every comparison here is exact equality of the f64
(or f32) arrays the reference would produce.
"""

import numpy as np
import pytest

from oracle import scipp_semantics as ora

pytestmark = pytest.mark.gpu

STRATEGIES = ['atomic', 'partition', 'paged', 'split', 'pixel', 'wide']

# internal kernel variants that must all be bit-identical
VARIANTS = [
    {},
    {'LDE_LUT32': '1'},
    {'LDE_TOA_GENERAL': '1'},
    {'LDE_TILE_BITS': '15', 'LDE_PART_GRID': '7'},
    # SPLIT: few hot rows (mostly cold keys), few split blocks (long cold regions),
    # hot set re-selected every batch
    {'LDE_HOT_ROWS': '8', 'LDE_SPLIT_GRID': '3', 'LDE_HOT_REFRESH': '1'},
    # SPLIT pixel table: tiny (constant tag conflicts), large
    {'LDE_PIXEL_CACHE_BITS': '11', 'LDE_SPLIT_GRID': '17'},
    {'LDE_PIXEL_CACHE_BITS': '15'},
    # SIEVE with few hot rows and few blocks: long cold regions, many sort
    # pieces per wave, tiles split over several accumulate items
    {'LDE_HOT_ROWS': '8', 'LDE_SPLIT_GRID': '3', 'LDE_ITEM_EVENTS': '40000'},
    # one sieve block: its chunk range exceeds the LDS chunk table (global table)
    {'LDE_SPLIT_GRID': '1'},
]


@pytest.fixture(scope='module', autouse=True)
def _gpu(engine_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip('no HIP device')


def _engine(view, edges_ns, strategy='auto', **kw):
    from esslivedata_amd.engine import BinningEngine

    return BinningEngine(
        toa_edges_ns=edges_ns,
        out_lut=view.lut,
        pid_offset=view.pid_offset,
        n_screen=view.n_screen,
        strategy=strategy,
        **kw,
    )


def _oracle_pixel_screen_geometric(inst):
    edges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    r = next(iter(inst.coords.values())).shape[0]
    return np.stack([ora.geometric_screen_index(inst.coords, edges, k) for k in range(r)])


# ---------------------------------------------------------------------------
def test_monitor_kat_reference_fixture():
    """monitor_workflow_test.py:176-183: TOA 1..5 ns, edges linspace(0,10,6) ns."""
    from esslivedata_amd.engine import BinningEngine

    edges = np.linspace(0, 10, 6)
    eng = BinningEngine.monitor(edges)
    eng.stage(None, np.array([1, 2, 3, 4, 5], dtype=np.int32))
    eng.accumulate()
    res = eng.finalize(hists=True)
    np.testing.assert_array_equal(res.current_hist.ravel(), [1, 2, 2, 0, 0])
    assert res.current_total == 5
    np.testing.assert_array_equal(
        res.current_hist.ravel(), ora.monitor_histogram(np.arange(1, 6), edges)
    )


MONITOR_VARIANTS = [{}]


@pytest.mark.parametrize('layout', ['large', 'small'])
@pytest.mark.parametrize('variant', range(len(MONITOR_VARIANTS)))
@pytest.mark.parametrize('n_bins', [100, 7, 1000, 3000, 10000])
def test_monitor_matches_oracle(n_bins, variant, layout, request):
    """Several messages per launch, message sizes not multiples of 4 or of
    the grid; each message gets its own range of blocks."""
    from esslivedata_amd.engine import BinningEngine

    if MONITOR_VARIANTS[variant]:  # the diagnostics build reads the knobs
        request.getfixturevalue('knobs')(**MONITOR_VARIANTS[variant])
    rng = np.random.default_rng(n_bins)
    edges = np.geomspace(0.5, 71.43, n_bins + 1) * 1e6
    toa = np.concatenate(
        [
            rng.normal(30e6, 10e6, 200_000).astype(np.int32),
            np.ceil(edges).astype(np.int32),
            np.ceil(edges).astype(np.int32) - 1,
            np.full(50_000, int(np.ceil(edges[3])), dtype=np.int32),  # hot bin
        ]
    )
    eng = BinningEngine.monitor(edges)
    # three messages: large, or one of 3 events (its block range holds one block)
    cuts = (0, 100_000, 180_000) if layout == 'large' else (0, 3, 100_003)
    for lo, hi in zip(cuts, cuts[1:] + (len(toa),)):
        eng.stage(None, toa[lo:hi])
    eng.accumulate()
    res = eng.finalize(hists=True)
    np.testing.assert_array_equal(res.current_hist.ravel(), ora.monitor_histogram(toa, edges))


@pytest.mark.parametrize('strategy', STRATEGIES)
def test_dummy_logical_view_multi_batch(strategy):
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dummy_panel()
    view = projection.logical_lut(inst.detector_number, dims=('y', 'x'))
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, strategy)
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=ora.logical_screen_index(inst.detector_number.shape, None)[0][None, :],
        screen_shape=(128, 128),
        toa_edges_ns=edges,
    )
    for batch, size in enumerate([2000, 3000, 1000, 1000, 250_000]):
        pid, toa = synthetic.fake_detector_events(size, 0, 16384 + 5, seed=batch)
        eng.stage(pid, toa)
        eng.accumulate(0)
        o.accumulate(pid, toa)
        if batch in (0, 1, 3, 4):
            res = eng.finalize(hists=True)
            exp = o.finalize()
            np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
            np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
            np.testing.assert_array_equal(res.current_image.reshape(128, 128), exp['current'])
            np.testing.assert_array_equal(
                res.cumulative_image.reshape(128, 128), exp['cumulative']
            )
            assert res.current_total == exp['counts_total']
            assert res.cumulative_total == exp['counts_total_cumulative']


@pytest.mark.parametrize('variant', range(len(VARIANTS)))
@pytest.mark.parametrize('strategy', STRATEGIES)
def test_dream_mantle_geometric_skewed(strategy, variant, knobs):
    knobs(**VARIANTS[variant])
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    lo, hi = 10, 90
    eng = _engine(view, edges, strategy, toa_range=(lo, hi))
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=_oracle_pixel_screen_geometric(inst),
        screen_shape=(80, 320),
        toa_edges_ns=edges,
        toa_slice=(lo, hi),
    )
    for batch in range(3):  # replicas cycle 0, 1, 2
        pid, toa = synthetic.dream_events(1_500_000, inst, seed=100 + batch)
        # unknown ids on both sides of the LUT
        pid[:1000] = 229376
        pid[1000:2000] = 720897
        eng.stage(pid[: len(pid) // 2], toa[: len(toa) // 2])
        eng.stage(pid[len(pid) // 2 :], toa[len(toa) // 2 :])
        eng.accumulate(batch % view.n_replicas)
        o.accumulate(pid, toa)
    res = eng.finalize(hists=True)
    exp = o.finalize()
    # PIXEL needs footprints that fit LDS: the mantle's 2048-pixel ranges span
    # two arc columns of 320 screens, so it falls back to WIDE here; so does
    # SPLIT on the general TOA layout (the sieve bins through the fast one)
    fallback = strategy == 'pixel' or (strategy == 'split' and 'LDE_TOA_GENERAL' in VARIANTS[variant])
    assert eng.info()['last_strategy'] == ('wide' if fallback else strategy)
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
    np.testing.assert_array_equal(res.current_image.reshape(80, 320), exp['current'])
    assert res.current_in_range == exp['counts_in_toa_range']
    assert res.cumulative_in_range == exp['counts_in_toa_range_cumulative']


@pytest.mark.parametrize('general', [False, True])
@pytest.mark.parametrize('strategy', STRATEGIES)
def test_edge_ties_are_bit_exact(strategy, general, knobs):
    """Integer TOAs on, just below and just above every float64 edge."""
    if general:
        knobs(LDE_TOA_GENERAL='1')
    from esslivedata_amd import projection

    dn = np.arange(1, 65, dtype=np.int32)
    view = projection.logical_lut(dn)
    for edges in (
        np.linspace(0, 71.43, 101) * 1e6,
        np.geomspace(0.5, 71.43, 101) * 1e6,
        np.array([-5.5, -0.5, 0.0, 0.5, 1.0, 1.0, 2.5, 3.0, 1e6 + 0.25]),
        np.array([-3e9, -2.0**31, -1.5, 7.0, 2.0**31 - 1, 2.0**31, 5e9]),
        np.array([10.0, 10.0, 10.0]),
        np.sort(np.random.default_rng(3).uniform(-1e5, 1e5, 2001)),
    ):
        c = np.ceil(edges).astype(np.int64)
        toa = np.concatenate([c - 1, c, c + 1, np.floor(edges).astype(np.int64)])
        toa = np.clip(toa, -(2**31), 2**31 - 1).astype(np.int32)
        pid = np.resize(dn, len(toa))
        eng = _engine(view, edges, strategy)
        eng.stage(pid, toa)
        eng.accumulate(0)
        got = eng.finalize(hists=True).current_hist
        pix = ora.pixel_index(pid, dn)
        exp = ora.detector_histogram(np.arange(64), 64, pix, toa, edges)
        np.testing.assert_array_equal(got, exp)


def test_bifrost_float32_accumulation():
    from esslivedata_amd import projection, synthetic

    inst = synthetic.bifrost_unified()
    view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'auto', out_dtype='float32')
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)[0][
            None, :
        ],
        screen_shape=(15, 900),
        toa_edges_ns=edges,
        dtype=np.float32,
    )
    for batch in range(20):
        pid, toa = synthetic.fake_detector_events(45_000, 1, 13500, seed=batch)
        eng.stage(pid, toa)
        eng.accumulate(0)
        o.accumulate(pid, toa)
        if batch % 5 == 4:
            res = eng.finalize(hists=True)
            exp = o.finalize()
            assert res.current_hist.dtype == np.float32
            np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
            np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])


@pytest.mark.parametrize('pushes', [1, 2, 5])
def test_bifrost_float32_fused_finalize_cadences(pushes):
    """float32 views keep a push's counts in the batch until the next
    accumulate or the finalize, which fuses its f32 adds (k_finalize_f32);
    one push per finalize is the reference cadence (core/job.py:413-433).
    Histogram reads, ROI-like group spectra and a clear between pushes merge
    the pending push first; every output equals the oracle's per-push float32
    sums, images over a TOA range included."""
    from esslivedata_amd import projection, synthetic

    inst = synthetic.bifrost_unified()
    view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'auto', out_dtype='float32', toa_range=(10, 90))
    ps = ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)[0][None, :]
    o = ora.OracleDetectorView(detector_number=inst.detector_number, pixel_screen=ps,
                               screen_shape=(15, 900), toa_edges_ns=edges, dtype=np.float32,
                               toa_slice=(10, 90))
    groups = [np.arange(0, 900), np.arange(450, 2000)]
    eng.set_groups(0, groups)
    for k in range(4 * pushes):
        pid, toa = synthetic.fake_detector_events(30_000 + 977 * k, 1, 13500, seed=300 + k)
        if k == 2 * pushes:  # a clear drops the window's pending push too
            eng.clear()
            o.clear()
        eng.stage(pid, toa)
        eng.accumulate(0)
        o.accumulate(pid, toa)
        if k % 3 == 1:  # reads between pushes see every push so far
            win = o._acc.window
            np.testing.assert_array_equal(eng.read_histogram('current'), win)
            np.testing.assert_array_equal(eng.read_histogram('cumulative'), o._acc.cumulative)
            sp = eng.group_spectra(0, 'current')
            np.testing.assert_array_equal(sp, np.stack([win[g].sum(0) for g in groups]))
        if k % pushes == pushes - 1:
            res = eng.finalize(images=True, hists=True)
            exp = o.finalize()
            assert res.current_hist.dtype == np.float32 and res.current_image.dtype == np.float32
            np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
            np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
            np.testing.assert_array_equal(res.current_image, exp['current'].ravel())
            np.testing.assert_array_equal(res.cumulative_image, exp['cumulative'].ravel())
            assert res.current_total == exp['counts_total']
            assert res.cumulative_in_range == exp['counts_in_toa_range_cumulative']


def test_atomic_many_large_messages_proportional_blocks():
    """More messages than fit the kernel arguments, large enough that their
    block ranges are shares of 8 blocks per CU (k_bin_atomic_blocks)."""
    import torch

    from esslivedata_amd import projection, synthetic

    inst = synthetic.bifrost_unified()
    view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'atomic')
    ps = ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)[0][None, :]
    o = ora.OracleDetectorView(detector_number=inst.detector_number, pixel_screen=ps,
                               screen_shape=(15, 900), toa_edges_ns=edges)
    pid, toa = synthetic.fake_detector_events(100 * 40_000, 1, 13500, seed=5)
    dp, dt = torch.as_tensor(pid, device='cuda'), torch.as_tensor(toa, device='cuda')
    sizes = np.random.default_rng(1).integers(1, 80_000, 100)
    bounds = np.minimum(np.concatenate([[0], np.cumsum(sizes)]), len(pid))
    eng.stage_tensors_batch([(dp[a:b], dt[a:b]) for a, b in zip(bounds[:-1], bounds[1:]) if b > a])
    eng.accumulate(0)
    n = int(bounds[-1])
    o.accumulate(pid[:n], toa[:n])
    res = eng.finalize(hists=True)
    np.testing.assert_array_equal(res.current_hist, o.finalize()['histogram_current'])


@pytest.mark.parametrize('n_msgs', [1, 24, 45, 64, 65, 130, 630])
def test_atomic_many_messages(n_msgs):
    """ATOMIC with many small messages per accumulate (BIFROST: 45 bank
    messages of 1,000 events per pulse): up to 64 descriptors per launch, or
    one descriptor per block past that (k_bin_atomic_blocks); messages of ragged
    sizes, some not 16-byte aligned, bit-exact against the oracle."""
    from esslivedata_amd import projection, synthetic

    inst = synthetic.bifrost_unified()
    view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'atomic')
    ps = ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)[0][None, :]
    o = ora.OracleDetectorView(detector_number=inst.detector_number, pixel_screen=ps,
                               screen_shape=(15, 900), toa_edges_ns=edges)
    import torch

    rng = np.random.default_rng(n_msgs)
    for batch in range(2):
        pid, toa = synthetic.fake_detector_events(1000 * n_msgs + 37, 1, 13500, seed=batch)
        dp = torch.as_tensor(pid, device='cuda')
        dt = torch.as_tensor(toa, device='cuda')
        cuts = np.sort(rng.choice(np.arange(1, len(pid)), n_msgs - 1, replace=False)) if n_msgs > 1 else []
        bounds = [0, *[int(c) for c in cuts], len(pid)]
        # one device segment per message (ragged, mostly misaligned)
        eng.stage_tensors_batch([(dp[a:b], dt[a:b]) for a, b in zip(bounds[:-1], bounds[1:])])
        eng.accumulate(0)
        o.accumulate(pid, toa)
        assert eng.info()['last_strategy'] == 'atomic'
        res = eng.finalize(hists=True)
        exp = o.finalize()
        np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
        np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])


def test_bifrost_float32_partials_match_finalize():
    """float32 views export their exact integer counts as partial outputs;
    rounded once to f32 they equal the handle's own f32 finalize images (every
    per-push f32 bin value is an exact integer here), over several windows."""
    import torch

    from esslivedata_amd import projection, synthetic

    inst = synthetic.bifrost_unified()
    view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    edges = inst.edges.edges_ns()
    a = _engine(view, edges, 'auto', out_dtype='float32', toa_range=(10, 90))
    b = _engine(view, edges, 'auto', out_dtype='float32', toa_range=(10, 90))
    S = view.n_screen
    buf = torch.zeros(2 * S + 4, dtype=torch.int64, device='cuda')
    for batch in range(12):
        pid, toa = synthetic.fake_detector_events(45_000, 1, 13500, seed=100 + batch)
        for e in (a, b):
            e.stage(pid, toa)
            e.accumulate(0)
        if batch % 4 == 3:
            ref = a.finalize(images=True)
            b.finalize_partials(buf.data_ptr())
            b.synchronize()
            h = buf.cpu().numpy()
            assert ref.current_image.dtype == np.float32
            np.testing.assert_array_equal(h[:S].astype(np.float32), ref.current_image)
            np.testing.assert_array_equal(h[S:2 * S].astype(np.float32), ref.cumulative_image)
            assert [int(x) for x in h[2 * S:]] == [ref.current_total, ref.current_in_range,
                                                   ref.cumulative_total, ref.cumulative_in_range]
    # the f32 window restarted after the partials: b's next finalize = a's
    pid, toa = synthetic.fake_detector_events(45_000, 1, 13500, seed=999)
    for e in (a, b):
        e.stage(pid, toa)
        e.accumulate(0)
    ra, rb = a.finalize(hists=True), b.finalize(hists=True)
    np.testing.assert_array_equal(ra.current_hist, rb.current_hist)
    np.testing.assert_array_equal(ra.cumulative_hist, rb.cumulative_hist)


def test_empty_and_all_dropped_batches():
    from esslivedata_amd import projection

    dn = np.arange(10, 20, dtype=np.int32)
    view = projection.logical_lut(dn)
    edges = np.linspace(0, 100, 11)
    eng = _engine(view, edges)
    with pytest.raises(ValueError, match='No data'):
        eng.finalize()
    eng.accumulate(0)  # empty batch still produces (zero) outputs
    res = eng.finalize(hists=True)
    assert res.current_total == 0 and res.cumulative_total == 0
    eng.stage(np.array([1, 2, 30], np.int32), np.array([5, 5, 5], np.int32))  # unknown ids
    eng.stage(np.array([10, 11], np.int32), np.array([-1, 100], np.int32))  # out of range TOA
    eng.accumulate(0)
    res = eng.finalize(hists=True)
    assert res.current_total == 0
    with pytest.raises(ValueError):
        eng.accumulate(1)  # replica out of range
    with pytest.raises(ValueError):
        eng.stage(np.array([1, 2], np.int32), np.array([1], np.int32))


def test_reset_and_clear_semantics():
    from esslivedata_amd import projection

    dn = np.arange(1, 5, dtype=np.int32)
    view = projection.logical_lut(dn)
    edges = np.linspace(0, 10, 3)
    eng = _engine(view, edges)
    eng.stage(np.array([1, 2], np.int32), np.array([1, 6], np.int32))
    eng.accumulate(0)
    eng.finalize()
    eng.stage(np.array([3], np.int32), np.array([1], np.int32))
    eng.accumulate(0)
    assert eng.read_histogram('cumulative').sum() == 3
    eng.reset_cumulative()  # geometry changed: drop cumulative and window
    eng.stage(np.array([4], np.int32), np.array([7], np.int32))
    eng.accumulate(0)
    res = eng.finalize(hists=True)
    assert res.cumulative_total == 1 and res.current_total == 1
    eng.clear()
    with pytest.raises(ValueError):
        eng.finalize()


@pytest.mark.parametrize('strategy', STRATEGIES)
def test_device_staging_matches_host_staging(strategy):
    import torch

    from esslivedata_amd import projection, synthetic

    inst = synthetic.loki_bank0()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution, flip_x=True)
    edges = inst.edges.edges_ns()
    pid, toa = synthetic.uniform_events(3_000_001, 1, 802816 + 100, seed=5)
    a = _engine(view, edges, strategy)
    a.stage(pid, toa)
    a.accumulate(1)
    b = _engine(view, edges, strategy)
    dp = torch.as_tensor(pid, device='cuda')
    dt = torch.as_tensor(toa, device='cuda')
    b.stage_tensors(dp[:1_000_003], dt[:1_000_003])  # misaligned second segment
    b.stage_tensors(dp[1_000_003:], dt[1_000_003:])
    b.accumulate(1)
    np.testing.assert_array_equal(a.read_histogram(), b.read_histogram())
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=_oracle_pixel_screen_geometric(
            synthetic.Instrument(
                'l', inst.detector_number, {'x': -inst.coords['x'], 'y': inst.coords['y']},
                inst.resolution, inst.edges,
            )
        ),
        screen_shape=(144, 144),
        toa_edges_ns=edges,
    )
    np.testing.assert_array_equal(a.read_histogram(), o.batch_histogram(pid, toa, 1))
    # the same batch through lde_stage_device_batch (one call, an empty message in it)
    c = _engine(view, edges, strategy)
    cuts = [0, 7, 1_000_003, 1_000_003, 2_500_000, len(pid)]
    c.stage_tensors_batch([(dp[x:y], dt[x:y]) for x, y in zip(cuts[:-1], cuts[1:])])
    c.accumulate(1)
    np.testing.assert_array_equal(a.read_histogram(), c.read_histogram())
    with pytest.raises(ValueError):
        c.stage_tensors_batch([(dp[:5], dt[:4])])


def test_auto_picks_split_for_skewed_and_pixel_for_uniform():
    """AUTO: the sampled hot-row coverage decides SPLIT; an unskewed stream whose
    pixel-range footprints fit in LDS takes PIXEL (performance only; counts exact)."""
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges)
    pid, toa = synthetic.dream_events(3_000_000, inst, seed=11)
    eng.stage(pid, toa)
    eng.accumulate(3)
    assert eng.info()['last_strategy'] == 'split'
    exp = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=_oracle_pixel_screen_geometric(inst),
        screen_shape=(80, 320),
        toa_edges_ns=edges,
    ).batch_histogram(pid, toa, 3)
    np.testing.assert_array_equal(eng.read_histogram(), exp)

    inst = synthetic.loki_bank0()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    eng = _engine(view, inst.edges.edges_ns())
    pid, toa = synthetic.uniform_events(3_000_000, 1, 802816, seed=5)
    eng.stage(pid, toa)
    eng.accumulate(0)
    assert eng.info()['last_strategy'] == 'pixel'
    exp = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=_oracle_pixel_screen_geometric(inst),
        screen_shape=view.screen_shape,
        toa_edges_ns=inst.edges.edges_ns(),
    ).batch_histogram(pid, toa, 0)
    np.testing.assert_array_equal(eng.read_histogram(), exp)


def test_finalize_partials_match_finalize():
    """lde_finalize_partials (multi-GPU outputs) == lde_finalize, over batches,
    including an empty window (a rank that received no events)."""
    import torch

    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    a = _engine(view, edges)
    b = _engine(view, edges)
    S = view.n_screen
    buf = torch.zeros(2 * S + 4, dtype=torch.int64, device='cuda')
    for batch, n in enumerate([300_000, 0, 2_000_000]):
        pid, toa = synthetic.dream_events(n, inst, seed=30 + batch)
        if n:
            a.stage(pid, toa)
            a.accumulate(batch % view.n_replicas)
            b.stage(pid, toa)
            b.accumulate(batch % view.n_replicas)
            ref = a.finalize(images=True)
        b.finalize_partials(buf.data_ptr())
        b.synchronize()  # b runs on its own stream
        h = buf.cpu().numpy()
        if n:
            np.testing.assert_array_equal(h[:S].astype(np.float64), ref.current_image)
            np.testing.assert_array_equal(h[S:2 * S].astype(np.float64), ref.cumulative_image)
            assert [int(x) for x in h[2 * S:]] == [ref.current_total, ref.current_in_range,
                                                   ref.cumulative_total, ref.cumulative_in_range]
        else:
            assert not h[:S].any() and int(h[2 * S]) == 0 and int(h[2 * S + 2]) > 0


@pytest.mark.parametrize('grid', ['8', '17'])
def test_sieve_few_blocks_ragged_messages(grid, knobs):
    """Few sieve blocks (long chunk ranges, chunk tables in LDS) over ragged
    device messages (partial and misaligned chunks inside the ranges), three
    batches on rotating replicas, bit-exact against the oracle."""
    import torch

    knobs(LDE_SPLIT_GRID=grid)
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'split')
    o = ora.OracleDetectorView(detector_number=inst.detector_number,
                               pixel_screen=_oracle_pixel_screen_geometric(inst),
                               screen_shape=(80, 320), toa_edges_ns=edges)
    rng = np.random.default_rng(int(grid))
    for batch in range(3):
        pid, toa = synthetic.dream_events(2_400_007 + batch, inst, seed=400 + batch)
        dp = torch.as_tensor(pid, device='cuda')
        dt = torch.as_tensor(toa, device='cuda')
        cuts = np.sort(rng.choice(np.arange(1, len(pid)), 6, replace=False))
        bounds = [0, *cuts.tolist(), len(pid)]
        eng.stage_tensors_batch([(dp[a:b], dt[a:b]) for a, b in zip(bounds[:-1], bounds[1:])])
        eng.accumulate(batch % view.n_replicas)
        o.accumulate(pid, toa)
        assert eng.info()['last_strategy'] == 'split'
    res = eng.finalize(hists=True)
    exp = o.finalize()
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])


@pytest.mark.parametrize('n_msgs', [1, 14, 24, 25, 40])
def test_split_many_device_messages(n_msgs, knobs):
    """SIEVE with the message descriptors passed as kernel arguments (<= 24
    messages) or uploaded (more): ragged, misaligned device segments, replica
    cycling, hot-set refresh every other batch."""
    import torch

    knobs(LDE_HOT_REFRESH='2')
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'split')
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=_oracle_pixel_screen_geometric(inst),
        screen_shape=(80, 320),
        toa_edges_ns=edges,
    )
    rng = np.random.default_rng(n_msgs)
    for batch in range(3):
        pid, toa = synthetic.dream_events(1_000_003, inst, seed=200 + batch)
        dp = torch.as_tensor(pid, device='cuda')
        dt = torch.as_tensor(toa, device='cuda')
        cuts = np.sort(rng.choice(np.arange(1, len(pid)), n_msgs - 1, replace=False))
        bounds = [0, *cuts.tolist(), len(pid)]
        eng.stage_tensors_batch([(dp[a:b], dt[a:b]) for a, b in zip(bounds[:-1], bounds[1:])])
        eng.accumulate(batch % view.n_replicas)
        o.accumulate(pid, toa)
    res = eng.finalize(hists=True)
    exp = o.finalize()
    assert eng.info()['last_strategy'] == 'split'
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])


def test_side_stream_producer_is_ordered_and_kept_alive():
    """events produced on another torch stream with a
    non-blocking copy behind a slow kernel, staged, and dropped right after
    accumulate while new allocations on that stream reuse their blocks.  The
    engine (own stream) must wait for the producer and the allocator must not
    hand the blocks out before the engine's kernels are done."""
    import torch

    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    o = ora.OracleDetectorView(detector_number=inst.detector_number,
                               pixel_screen=_oracle_pixel_screen_geometric(inst),
                               screen_shape=(80, 320), toa_edges_ns=edges)
    for strategy in ('split', 'atomic'):
        eng = _engine(view, edges, strategy)  # engine-owned stream
        side = torch.cuda.Stream()
        slow = torch.randn(4096, 4096, device='cuda')
        for batch in range(3):
            pid, toa = synthetic.dream_events(2_000_000 if strategy == 'split' else 200_000, inst,
                                              seed=300 + batch)
            hp = torch.from_numpy(pid).pin_memory()
            ht = torch.from_numpy(toa).pin_memory()
            with torch.cuda.stream(side):
                for _ in range(8):  # keep the producer stream busy
                    slow = slow @ slow
                    slow /= slow.abs().max()
                dp = hp.to('cuda', non_blocking=True)
                dt = ht.to('cuda', non_blocking=True)
                if batch == 2:
                    eng.stage_tensors_batch([(dp[:777], dt[:777]), (dp[777:], dt[777:])])
                else:
                    eng.stage_tensors(dp, dt)
                del dp, dt
                eng.accumulate(batch)
                junk = [torch.full((len(pid),), -5, dtype=torch.int32, device='cuda')
                        for _ in range(4)]  # may reuse the staged blocks
                del junk
            got = eng.finalize(hists=True).current_hist
            np.testing.assert_array_equal(got, o.batch_histogram(pid, toa, batch))
        eng.close()


def test_device_tensors_must_be_int32():
    """float32 / uint32 / int64 tensors are refused, not
    reinterpreted as int32 bits."""
    import torch

    from esslivedata_amd import projection

    dn = np.arange(1, 65, dtype=np.int32)
    view = projection.logical_lut(dn)
    eng = _engine(view, np.linspace(0, 100, 11))
    ok = torch.arange(10, dtype=torch.int32, device='cuda')
    for bad in (torch.float32, torch.int64, torch.uint32, torch.int16):
        b = torch.arange(10, device='cuda').to(bad)
        with pytest.raises(ValueError):
            eng.stage_tensors(ok, b)
        with pytest.raises(ValueError):
            eng.stage_tensors(b, ok)
        with pytest.raises(ValueError):
            eng.stage_tensors_batch([(ok, ok), (b, ok)])
    with pytest.raises(ValueError):
        eng.stage_tensors(ok.cpu(), ok.cpu())
    assert eng.info()['staged'] == 0


def test_default_stream_engine_outlives_recorded_tensors():
    """An engine on its default (torch pool) stream, fed from torch's null
    stream, then destroyed before the staged tensors are freed: the caching
    allocator's stream record must point at a live stream (the round-2
    regression: record_stream on an engine-destroyed stream crashed at free)."""
    import torch

    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle(n_replicas=1)
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    pid, toa = synthetic.dream_events(500_000, inst, seed=8)
    dp = torch.as_tensor(pid, device='cuda')
    dt = torch.as_tensor(toa, device='cuda')
    eng = _engine(view, inst.edges.edges_ns())
    assert eng.stream_ptr != torch.cuda.current_stream().cuda_stream
    eng.stage_tensors_batch([(dp[:1000], dt[:1000]), (dp[1000:], dt[1000:])])
    eng.accumulate(0)
    h = eng.read_histogram()
    eng.close()
    del eng, dp, dt
    torch.cuda.synchronize()
    x = torch.empty(10**7, dtype=torch.int32, device='cuda')  # allocator reuse after free
    del x
    assert h.sum() > 0


@pytest.mark.parametrize('grid', ['1', '3'])
def test_sieve_hot_cells_with_millions_of_events(grid, knobs):
    """One or three sieve blocks (one: its chunk range exceeds the LDS chunk
    table); two adjacent hot cells take 1.8 M and 0.6 M events per batch,
    far past any 16-bit count, plus a third hot screen and a uniform rest."""
    knobs(LDE_SPLIT_GRID=grid)
    from esslivedata_amd import projection

    dn = np.arange(1, 4097, dtype=np.int32)
    view = projection.logical_lut(dn)
    edges = np.linspace(0.0, 71.43, 101) * 1e6
    rng = np.random.default_rng(5)
    n = 3_000_000
    pid = rng.integers(1, 4097, n).astype(np.int32)
    toa = rng.uniform(0, 71e6, n).astype(np.int32)
    mid = lambda b: int((edges[b] + edges[b + 1]) / 2)  # noqa: E731
    k = rng.random(n)
    pid[k < 0.8] = 7
    toa[k < 0.6] = mid(10)
    toa[(k >= 0.6) & (k < 0.8)] = mid(11)
    pid[(k >= 0.8) & (k < 0.9)] = 8
    toa[(k >= 0.8) & (k < 0.9)] = mid(51)
    eng = _engine(view, edges, 'split')
    for _ in range(2):
        eng.stage(pid, toa)
        eng.accumulate(0)
    res = eng.finalize(hists=True)
    assert eng.info()['last_strategy'] == 'split'
    exp = 2 * ora.detector_histogram(np.arange(4096), 4096, ora.pixel_index(pid, dn), toa, edges)
    assert exp[6, 10] >= 2 * (k < 0.6).sum() > 3 * 65536
    np.testing.assert_array_equal(res.current_hist, exp)


def test_sieve_hot_rows_mixed_u16_and_u32_blocks(knobs):
    """Eight sieve blocks over one batch whose first half piles millions of
    events into two hot cells: the first blocks' hot rows overflow 16 bits
    (flushed as u32), the last blocks' do not (flushed as u16); the reduce
    mixes both formats."""
    knobs(LDE_SPLIT_GRID='8')
    from esslivedata_amd import projection

    dn = np.arange(1, 4097, dtype=np.int32)
    view = projection.logical_lut(dn)
    edges = np.linspace(0.0, 71.43, 101) * 1e6
    rng = np.random.default_rng(11)
    n = 4_000_000
    pid = rng.integers(1, 4097, n).astype(np.int32)
    toa = rng.uniform(0, 71e6, n).astype(np.int32)
    mid = lambda b: int((edges[b] + edges[b + 1]) / 2)  # noqa: E731
    head = np.arange(n) < n // 2
    k = rng.random(n)
    pid[head & (k < 0.7)] = 7
    toa[head & (k < 0.5)] = mid(10)
    toa[head & (k >= 0.5) & (k < 0.7)] = mid(11)
    pid[~head & (k < 0.3)] = 7  # still hot, but < 2^16 per block
    eng = _engine(view, edges, 'split')
    eng.stage(pid, toa)
    eng.accumulate(0)
    res = eng.finalize(hists=True)
    assert eng.info()['last_strategy'] == 'split'
    exp = ora.detector_histogram(np.arange(4096), 4096, ora.pixel_index(pid, dn), toa, edges)
    assert exp[6, 10] > 4 * 65536
    np.testing.assert_array_equal(res.current_hist, exp)


def test_finalize_images_written_in_place_are_never_reused_while_held():
    """Finalize images live in page-locked blocks the kernel writes directly;
    a block is handed out again only once the caller dropped every array (and
    view) of it, and past the pool cap finalize falls back to plain arrays."""
    from esslivedata_amd import projection

    dn = np.arange(1, 1025, dtype=np.int32)
    view = projection.logical_lut(dn)
    edges = np.linspace(0.0, 71.43, 11) * 1e6
    rng = np.random.default_rng(3)
    eng = _engine(view, edges, 'atomic')
    held, copies = [], []
    for k in range(12):
        pid = rng.integers(1, 1025, 5000 + 100 * k).astype(np.int32)
        toa = rng.uniform(0, 71e6, pid.size).astype(np.int32)
        eng.stage(pid, toa)
        eng.accumulate(0)
        res = eng.finalize(images=True)
        exp = ora.detector_histogram(np.arange(1024), 1024, ora.pixel_index(pid, dn), toa,
                                     edges).sum(axis=1)
        np.testing.assert_array_equal(res.current_image, exp)
        if k % 2 == 0:
            held.append(res.current_image[:])  # a view keeps its block
            copies.append(res.current_image.copy())
    for a, c in zip(held, copies):
        np.testing.assert_array_equal(a, c)
    ptrs = {a.__array_interface__['data'][0] for a in held}
    assert len(ptrs) == len(held)
    eng.close()


@pytest.mark.parametrize('strategy', ['pixel', 'paged', 'wide'])
def test_loki_pixel_ranges_multi_replica_and_move(strategy):
    """PIXEL (pixel-range partition, LUT slice in LDS) on LOKI bank 0 with
    five replicas, unknown ids, TOAs outside the edges, misaligned and empty
    messages, and a LUT replaced mid-run (a detector move rebuilds the
    footprints): bit-exact against the oracle, like PAGED."""
    from esslivedata_amd import geometry, projection, synthetic

    inst = synthetic.loki_bank0()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution, flip_x=True)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, strategy, toa_range=(5, 95))
    ps = ora.geometric_pixel_screen(inst.coords, inst.resolution, flip_x=True)
    o = ora.OracleDetectorView(detector_number=inst.detector_number, pixel_screen=ps,
                               screen_shape=(144, 144), toa_edges_ns=edges, toa_slice=(5, 95))
    for batch in range(4):
        if batch == 2:  # moved: new coordinates, new LUT, new footprints
            src = geometry.GeometricSource(inst.detector_number, inst.positions,
                                           projection_type='xy_plane', resolution=inst.resolution,
                                           pixel_noise=inst.pixel_noise, flip_x=True)
            t = np.eye(4)
            t[0, 3], t[1, 3] = 0.21, -0.13
            moved = src.view(t)
            eng.set_lut(moved.lut)
            o.pixel_screen = ora.geometric_pixel_screen(src.coords(t), inst.resolution, flip_x=True)
        pid, toa = synthetic.uniform_events(3_000_001 + batch, 1, 802816, seed=300 + batch)
        pid[:500] = 0  # unknown ids on both sides of the LUT
        pid[500:1000] = 802817
        toa[1000:1200] = -7  # before the first edge
        toa[1200:1400] = 2_000_000_000  # past the last edge
        eng.stage(pid[:1_000_001], toa[:1_000_001])
        eng.stage(pid[1_000_001:1_000_001], toa[1_000_001:1_000_001])
        eng.stage(pid[1_000_001:], toa[1_000_001:])
        eng.accumulate(batch % view.n_replicas)
        o.accumulate(pid, toa)
        res = eng.finalize(hists=True)
        exp = o.finalize()
        assert eng.info()['last_strategy'] == strategy
        np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
        np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
        assert res.current_in_range == exp['counts_in_toa_range']


def test_loki_pixel_forced_on_skewed_stream_splits_hot_ranges():
    """Forced PIXEL on a stream AUTO would not give it: 70 % of the events in
    the first 4,096 pixels (one pixel range) and a batch that is one pixel and
    one TOA value only.  A range holding many times the mean range total is
    split over several pass-B items whose footprint flushes add into the same
    bins; counts stay bit-exact."""
    from esslivedata_amd import projection, synthetic

    inst = synthetic.loki_bank0(n_replicas=1)
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'pixel')
    ps = _oracle_pixel_screen_geometric(inst)
    rng = np.random.default_rng(17)
    for batch in range(2):
        n = 8_000_003
        if batch == 0:
            pid, toa = synthetic.uniform_events(n, 1, 802816, seed=41)
            hot = rng.random(n) < 0.7
            pid[hot] = rng.integers(1, 4097, int(hot.sum())).astype(np.int32)
        else:
            pid = np.full(n, 123_457, dtype=np.int32)
            toa = np.full(n, 35_000_000, dtype=np.int32)
        eng.stage(pid, toa)
        eng.accumulate(0)
        res = eng.finalize(hists=True)
        assert eng.info()['last_strategy'] == 'pixel'
        exp = ora.detector_histogram(ps[0], view.n_screen, ora.pixel_index(pid, inst.detector_number),
                                     toa, edges)
        np.testing.assert_array_equal(res.current_hist, exp)
        assert res.current_total == int(exp.sum())


def test_loki_pixel_predicted_slots_exact_under_shifts(knobs):
    """PIXEL with predicted slots (no count pass: each (block, range) slot is
    sized from the previous batch's run totals).  Four partition blocks make
    the 784 slots hold >= 256 events each at 1e6 events per batch, so every
    batch after the first is predicted; the stream then shifts under the
    prediction: a new seed (a few runs past their slot), 70 % of the events
    in one pixel range, a 1.6x larger batch, one pixel only, and back.  Runs
    that miss their slot go through the overflow groups (global atomics);
    both replicas; counts stay bit-exact."""
    from esslivedata_amd import projection, synthetic

    knobs(LDE_PIX_GRID='4')
    inst = synthetic.loki_bank0(n_replicas=2)
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'pixel')
    ps = _oracle_pixel_screen_geometric(inst)
    rng = np.random.default_rng(23)
    cum = np.zeros((view.n_screen, len(edges) - 1), dtype=np.int64)
    for batch in range(7):
        n = 1_600_000 if batch == 4 else 1_000_000
        pid, toa = synthetic.uniform_events(n, 1, 802816, seed=100 + batch)
        if batch == 3:
            hot = rng.random(n) < 0.7
            pid[hot] = rng.integers(40_000, 44_096, int(hot.sum())).astype(np.int32)
        elif batch == 5:
            pid[:] = 654_321
        eng.stage(pid, toa)
        eng.accumulate(batch % 2)
        res = eng.finalize(hists=True)
        assert eng.info()['last_strategy'] == 'pixel'
        exp = ora.detector_histogram(ps[batch % 2], view.n_screen,
                                     ora.pixel_index(pid, inst.detector_number), toa, edges)
        cum += exp.astype(np.int64)
        np.testing.assert_array_equal(res.current_hist, exp)
        np.testing.assert_array_equal(res.cumulative_hist, cum)
        assert res.current_total == int(exp.sum())


PIXEL_VARIANTS = [
    {},
    # an overflow list of 16 groups: the overflow groups past it are added by
    # pass A itself (global atomics), exactly
    {'LDE_PIX_OVF_CAP': '16'},
]


@pytest.mark.parametrize('variant_knobs', PIXEL_VARIANTS, ids=lambda k: ','.join(f'{a}={b}' for a, b in k.items()) or 'default')
def test_loki_pixel_variants(knobs, variant_knobs):
    """Every PIXEL shape knob, counted (first batch) and predicted (second
    and third: six partition blocks, so 1.2e6-event batches fill the slots),
    bit-exact against the oracle over two replicas."""
    from esslivedata_amd import projection, synthetic

    knobs(LDE_PIX_GRID='6')
    knobs(**variant_knobs)
    inst = synthetic.loki_bank0(n_replicas=2)
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    eng = _engine(view, edges, 'pixel')
    ps = _oracle_pixel_screen_geometric(inst)
    for batch in range(3):
        pid, toa = synthetic.uniform_events(1_200_001 + 3 * batch, 1, 802816, seed=300 + batch)
        eng.stage(pid[: 500_000], toa[: 500_000])
        eng.stage(pid[500_000:], toa[500_000:])
        eng.accumulate(batch % 2)
        res = eng.finalize(hists=True)
        assert eng.info()['last_strategy'] == 'pixel'
        exp = ora.detector_histogram(ps[batch % 2], view.n_screen,
                                     ora.pixel_index(pid, inst.detector_number), toa, edges)
        np.testing.assert_array_equal(res.current_hist, exp)
