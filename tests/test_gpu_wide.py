"""GPU parity of the WIDE strategy: the reference's reachable TOA binnings.

``EdgesModel`` allows 1..10,000 bins, linear or log, from any start
(SRC/parameter_models.py:82-105, 290-295; the detector view's edges,
SRC/workflows/detector_view_specs.py:73-124).  Each test bins DREAM's mantle
(Zipf pixels, 5 noise replicas) or LOKI bank 0 (uniform pixels) at such a
binning, with AUTO choosing the strategy, and compares the full current and
cumulative (screen, TOA) histograms and the totals bit-exactly with
oracle/binning_ref.c run over the same events.  Small-size tests force the
two-level form, tiny and absent pixel tables, and views of 2 pixels.
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


def _setup(workload, num_bins, scale, start=None):
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle() if workload == 'dream' else synthetic.loki_bank0()
    inst = synthetic.with_toa_edges(inst, num_bins=num_bins, scale=scale, start=start)
    flip = workload == 'loki'
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution, flip_x=flip)
    ps = ora.geometric_pixel_screen(inst.coords, inst.resolution, flip_x=flip)
    return inst, view, ps


def _events(workload, inst, n, seed):
    from esslivedata_amd import synthetic

    if workload == 'dream':
        return synthetic.dream_events(n, inst, seed=seed)
    return synthetic.uniform_events(n, 1, 802816, seed=seed)


def _run(workload, num_bins, scale, start=None, n=30_000_000, strategy='auto', expect='wide', batches=2,
         toa_range=None):
    """Two batches of n events (replicas 0 and 1) with a finalize after each,
    as device messages of unequal sizes; every output against the C oracle."""
    import torch

    from esslivedata_amd.engine import BinningEngine
    from oracle import c_oracle

    inst, view, ps = _setup(workload, num_bins, scale, start)
    edges = inst.edges.edges_ns()
    kw = {'toa_range': toa_range} if toa_range else {}
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy, **kw)
    cur = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, edges)
    cum = np.zeros(view.n_screen * num_bins, dtype=np.int64)
    for b in range(batches):
        pid, toa = _events(workload, inst, n, seed=40 + b)
        pid[:500] = view.pid_offset - 1  # unknown ids
        dp, dt = torch.as_tensor(pid, device='cuda'), torch.as_tensor(toa, device='cuda')
        cuts = [0, n // 7, n // 7 + 3, n // 2, n]  # ragged messages, one of 3 events
        eng.stage_tensors_batch([(dp[a:c], dt[a:c]) for a, c in zip(cuts, cuts[1:])])
        eng.accumulate(b % view.n_replicas)
        assert eng.info()['last_strategy'] == expect
        res = eng.finalize(hists=True)
        cur.hist[:] = 0
        cur.accumulate(pid, toa, b % view.n_replicas)
        ref = cur.hist.astype(np.int64)
        cum += ref
        shape = (view.n_screen, num_bins)
        np.testing.assert_array_equal(res.current_hist, ref.reshape(shape).astype(np.float64))
        np.testing.assert_array_equal(res.cumulative_hist, cum.reshape(shape).astype(np.float64))
        assert res.current_total == int(ref.sum())
        assert res.cumulative_total == int(cum.sum())
        del dp, dt
    eng.close()


# DREAM mantle (Zipf, 5 replicas) at 3e7 events per batch: the sizes the
# verdict of round 5 asked for, log (the instrument's) and linear edges, and
# a log range starting at 0.01 ms (bins of 89 ns at the start)
@pytest.mark.parametrize('num_bins,scale,start', [
    (164, 'log', None), (1000, 'log', None), (1000, 'linear', None), (1000, 'log', 0.01),
    (10000, 'log', None), (10000, 'linear', None)])
def test_dream_wide_toa_binnings(num_bins, scale, start):
    _run('dream', num_bins, scale, start)


@pytest.mark.parametrize('num_bins,scale,start', [
    (164, 'linear', None), (1000, 'linear', None), (1000, 'log', 0.01), (10000, 'linear', None)])
def test_loki_wide_toa_binnings(num_bins, scale, start):
    _run('loki', num_bins, scale, start)


def test_dream_wide_toa_range_images():
    """Images and in-range totals over a TOA slice of a 1000-bin view."""
    import torch

    from esslivedata_amd.engine import BinningEngine

    inst, view, ps = _setup('dream', 1000, 'log')
    edges = inst.edges.edges_ns()
    lo, hi = 100, 900
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, toa_range=(lo, hi))
    o = ora.OracleDetectorView(detector_number=inst.detector_number, pixel_screen=ps,
                               screen_shape=(80, 320), toa_edges_ns=edges, toa_slice=(lo, hi))
    for b in range(2):
        pid, toa = _events('dream', inst, 3_000_000, seed=70 + b)
        eng.stage_tensors_batch([(torch.as_tensor(pid, device='cuda'), torch.as_tensor(toa, device='cuda'))])
        eng.accumulate(b)
        o.accumulate(pid, toa)  # (replica = its batch counter, as the engine's b)
    assert eng.info()['last_strategy'] == 'wide'
    res = eng.finalize(images=True, hists=True)
    exp = o.finalize()
    np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
    np.testing.assert_array_equal(res.current_image.reshape(80, 320), exp['current'])
    np.testing.assert_array_equal(res.cumulative_image.reshape(80, 320), exp['cumulative'])
    assert res.current_in_range == exp['counts_in_toa_range']
    assert res.cumulative_in_range == exp['counts_in_toa_range_cumulative']


# WIDE's internal forms at small sizes (diagnostics build): the two-level
# form (bands of 2 tiles) on a view that fits one level, a pixel table of 16
# slots (constant tag conflicts) and none at all (every event gathers), many
# small first-pass blocks
WIDE_VARIANTS = [
    {'LDE_WIDE_LEVELS': '2'},
    {'LDE_WIDE_CACHE_BITS': '4'},
    {'LDE_WIDE_CACHE_BITS': '0'},
    {'LDE_WIDE_LEVELS': '2', 'LDE_WIDE_CACHE_BITS': '0'},
    # pass B's read-modify-write on a fresh window too (it stores otherwise)
    {'LDE_WIDE_WZERO': '0'},
]


@pytest.mark.parametrize('variant', range(len(WIDE_VARIANTS)))
@pytest.mark.parametrize('num_bins', [100, 1000])
def test_dream_wide_variants(variant, num_bins, knobs):
    knobs(**WIDE_VARIANTS[variant])
    _run('dream', num_bins, 'log', n=2_000_000, strategy='wide')


@pytest.mark.parametrize('n_pixels', [1, 2, 3, 5])
@pytest.mark.parametrize('strategy', ['wide', 'split', 'paged', 'atomic'])
def test_tiny_views(n_pixels, strategy):
    """Views of 1..5 pixels (a 2-pixel SPLIT view had a pixel
    table of 2 slots, which the sieve's 16-byte table copy skipped)."""
    from esslivedata_amd import projection
    from esslivedata_amd.engine import BinningEngine

    dn = np.arange(10, 10 + n_pixels, dtype=np.int32)
    view = projection.logical_lut(dn)
    edges = np.geomspace(0.5, 71.43, 101) * 1e6
    rng = np.random.default_rng(n_pixels)
    n = 300_000
    pid = rng.integers(8, 12 + n_pixels, n).astype(np.int32)  # some unknown ids
    toa = rng.normal(30e6, 10e6, n).astype(np.int32)
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy)
    eng.stage(pid, toa)
    eng.accumulate(0)
    got = eng.finalize(hists=True).current_hist
    exp = ora.detector_histogram(np.arange(n_pixels), n_pixels, ora.pixel_index(pid, dn), toa, edges)
    np.testing.assert_array_equal(got, exp)


def test_wide_counters_and_levels():
    """The form AUTO's WIDE takes for a view is visible through lde_counter."""
    from esslivedata_amd.engine import BinningEngine

    for num_bins, levels in ((1000, 1), (10000, 2)):
        inst, view, _ = _setup('dream', num_bins, 'log')
        eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut,
                            pid_offset=view.pid_offset, n_screen=view.n_screen)
        assert eng.counter('wide_levels') == levels
        assert eng.counter('wide_parts') <= 1024
        assert eng.counter('wide_tree_words') > 0
        eng.close()


def _random_edges(rng, kind):
    """Sorted float64 edges of the shapes the bucket tree must split: bin
    widths spread over nine decades, runs of equal edges, non-integer edges
    around integers, negative starts and spans past the int32 range."""
    n = int(rng.integers(2, 4000))
    if kind == 0:  # widths log-uniform from 1 ns to 1 s
        w = 10.0 ** rng.uniform(0, 9, n - 1)
        e = np.concatenate([[rng.uniform(-1e6, 1e6)], rng.uniform(-1e6, 1e6) + np.cumsum(w)])
    elif kind == 1:  # clustered: most edges within a few ns of a handful of points
        c = rng.uniform(-1e8, 1e8, 5)
        e = np.sort(rng.choice(c, n) + rng.normal(0, 3, n))
    elif kind == 2:  # duplicates and half-integers
        e = np.sort(np.round(rng.uniform(-5e4, 5e4, n) * 2) / 2)
        e[rng.integers(0, n, n // 4)] = e[0]
        e = np.sort(e)
    else:  # past the int32 range on both sides
        e = np.sort(rng.uniform(-6e9, 6e9, n))
    return np.sort(e.astype(np.float64))


@pytest.mark.parametrize('seed', range(12))
def test_wide_random_edges_match_oracle(seed):
    """Randomized TOA edges through WIDE's bucket tree (forced and AUTO on a
    2e6-event batch), TOAs drawn on, beside and between the edges; every bin
    against the NumPy oracle.  Parity unpinned beyond the oracle's restated
    scipp rule (`t` in bin i iff e[i] <= t < e[i+1])."""
    from esslivedata_amd import projection
    from esslivedata_amd.engine import BinningEngine

    rng = np.random.default_rng(1000 + seed)
    edges = _random_edges(rng, seed % 4)
    dn = np.arange(1, 257, dtype=np.int32)
    view = projection.logical_lut(dn)
    n = 2_000_000
    c = np.ceil(edges).astype(np.int64)
    toa = np.concatenate([
        rng.choice(np.concatenate([c - 1, c, c + 1]), n // 2),
        rng.uniform(edges[0] - 10, edges[-1] + 10, n - n // 2).astype(np.int64)])
    toa = np.clip(toa, -(2**31), 2**31 - 1).astype(np.int32)
    pid = rng.integers(0, 258, n).astype(np.int32)  # ids 0 and 257 unknown
    pix = ora.pixel_index(pid, dn)
    exp = ora.detector_histogram(np.arange(256), 256, pix, toa, edges)
    for strategy in ('wide', 'auto'):
        eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                            n_screen=view.n_screen, strategy=strategy)
        eng.stage(pid, toa)
        eng.accumulate(0)
        got = eng.finalize(hists=True).current_hist
        np.testing.assert_array_equal(got, exp)
        eng.close()


def test_split_cumulative_carries_past_2_32():
    """Views with wide rows keep the cumulative as u32 low words + high words
    (k_finalize_w4 moves 4 bytes per bin): windows imported as uint64 counts
    past 2^32 (lde_import_window_u64) force both carries, a low word that
    wraps and a window count with high bits; the cumulative histogram, its
    readback, group spectra and totals equal the exact uint64 sums."""
    import torch

    from esslivedata_amd import projection
    from esslivedata_amd.engine import BinningEngine

    dn = np.arange(1, 65, dtype=np.int32)
    view = projection.logical_lut(dn)
    T = 200
    edges = np.linspace(0, 71.43, T + 1) * 1e6
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen)
    rng = np.random.default_rng(5)
    n = 64 * T
    cum = np.zeros(n, dtype=np.uint64)
    eng.set_groups(0, [np.arange(0, 64, 2), np.arange(10, 20), np.array([63])])
    for step in range(4):
        w = rng.integers(0, 2**32, n, dtype=np.uint64)
        w[rng.integers(0, n, n // 3)] = 0  # empty groups too
        w[:8] = 2**32 - 1  # low words wrap from the second window on
        w[8:16] = np.uint64(2**33 + 7)  # counts with high bits
        d = torch.as_tensor(w.view(np.int64), device='cuda')
        eng.import_window_u64(d.data_ptr())
        torch.cuda.synchronize()
        cum += w
        res = eng.finalize(images=True, hists=True)
        np.testing.assert_array_equal(res.cumulative_hist.ravel(), cum.astype(np.float64))
        assert res.cumulative_total == int(cum.sum(dtype=np.uint64))
        np.testing.assert_array_equal(
            res.cumulative_image, cum.reshape(64, T).sum(axis=1, dtype=np.uint64).astype(np.float64))
    np.testing.assert_array_equal(eng.read_histogram('cumulative').ravel(), cum.astype(np.float64))
    spec = eng.group_spectra(0, 'cumulative')
    c2 = cum.reshape(64, T)
    exp = np.stack([c2[0:64:2].sum(0, dtype=np.uint64), c2[10:20].sum(0, dtype=np.uint64), c2[63]])
    np.testing.assert_array_equal(spec, exp.astype(np.float64))
    eng.close()


def test_wide_hot_dropped_pixels_under_the_last_tag():
    """A view of 2^22 pixels keeps WIDE's 2^13-slot pixel table with tags up
    to 511; hot pixels with no screen (LUT -1) whose table words carry tag 511
    must stay dropped (their word once equalled the front end's 'no word'
    marker, which would have sent them to screen 0)."""
    from esslivedata_amd.engine import BinningEngine

    L, S = 1 << 22, 1000
    lut = (np.arange(L, dtype=np.int64) % S).astype(np.int32)
    hot = np.arange(4_190_000, 4_190_064)
    lut[hot] = -1
    lut[5:9] = -1  # dropped pixels under tag 0 as well
    edges = np.geomspace(0.5, 71.43, 1001) * 1e6
    rng = np.random.default_rng(11)
    n = 3_000_000
    pid = np.where(rng.random(n) < 0.5, rng.choice(hot, n), rng.integers(0, L, n)).astype(np.int32)
    toa = rng.uniform(0.4e6, 72e6, n).astype(np.int32)
    exp = ora.detector_histogram(lut, S, pid.astype(np.int64), toa, edges)
    for strategy in ('wide', 'auto'):
        eng = BinningEngine(toa_edges_ns=edges, out_lut=lut, pid_offset=0, n_screen=S, strategy=strategy)
        eng.stage(pid, toa)
        eng.accumulate(0)
        assert eng.info()['last_strategy'] == 'wide'
        got = eng.finalize(hists=True).current_hist
        np.testing.assert_array_equal(got, exp)
        eng.close()


def test_wide_windows_with_mixed_strategies():
    """Windows whose batches take different strategies (WIDE, then a small
    batch on ATOMIC in the same window): the fresh-window store-only flush,
    the read-modify-write flush and the per-screen cumulative sums across
    them.  Three windows at 1,000 bins: WIDE only, WIDE + ATOMIC, WIDE only;
    current and cumulative histograms against the C oracle."""
    import torch

    from esslivedata_amd.engine import BinningEngine
    from oracle import c_oracle

    inst, view, ps = _setup('dream', 1000, 'log')
    edges = inst.edges.edges_ns()
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen)
    cur = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, edges)
    cum = np.zeros(view.n_screen * 1000, dtype=np.int64)
    plan = [[2_000_000], [2_000_000, 50_000], [1_500_000]]
    seed = 300
    for w, sizes in enumerate(plan):
        cur.hist[:] = 0
        strategies = []
        for n in sizes:
            pid, toa = synthetic_events(inst, n, seed)
            seed += 1
            eng.stage_tensors_batch([(torch.as_tensor(pid, device='cuda'), torch.as_tensor(toa, device='cuda'))])
            eng.accumulate(0)
            strategies.append(eng.info()['last_strategy'])
            cur.accumulate(pid, toa, 0)
        assert strategies[0] == 'wide' and (len(sizes) == 1 or strategies[1] == 'atomic')
        res = eng.finalize(hists=True)
        ref = cur.hist.astype(np.int64)
        cum += ref
        np.testing.assert_array_equal(res.current_hist.ravel(), ref.astype(np.float64))
        np.testing.assert_array_equal(res.cumulative_hist.ravel(), cum.astype(np.float64))
        assert res.current_total == int(ref.sum())
    eng.close()


def synthetic_events(inst, n, seed):
    from esslivedata_amd import synthetic

    return synthetic.dream_events(n, inst, seed=seed)


def test_wide_float32_view_per_push_sums():
    """A float32 view (BIFROST's unified view) at 1,000 TOA bins: batches of
    2e6 events take WIDE, and the per-push float32 window and cumulative sums
    equal the oracle's (the fresh-window store-only flush and the split
    cumulative are integer-view forms; this view keeps the exact u64 one)."""
    from esslivedata_amd import projection, synthetic

    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.bifrost_unified()
    view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    edges = np.geomspace(0.5, 71.43, 1001) * 1e6
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, out_dtype='float32')
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number,
        pixel_screen=ora.logical_screen_index((5, 3, 9, 100), synthetic.bifrost_transform)[0][None, :],
        screen_shape=(15, 900), toa_edges_ns=edges, dtype=np.float32)
    for batch in range(4):
        pid, toa = synthetic.fake_detector_events(2_000_000, 1, 13500, seed=500 + batch)
        eng.stage(pid, toa)
        eng.accumulate(0)
        assert eng.info()['last_strategy'] == 'wide'
        o.accumulate(pid, toa)
        if batch % 2 == 1:
            res = eng.finalize(hists=True)
            exp = o.finalize()
            assert res.current_hist.dtype == np.float32
            np.testing.assert_array_equal(res.current_hist, exp['histogram_current'])
            np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
    eng.close()
