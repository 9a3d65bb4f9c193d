"""The split finalize (images and totals from the window's rows; the fold of
the window into the cumulative histogram queued behind the host's wake-up
event) against the CPU oracle, bit-exact, across the state changes that touch
the cumulative histogram: a finalize with histograms (the single-kernel path,
after which the running row sums are rebuilt) and reset_cumulative.  Windows
folded into u64 (past 2^32 events per window) are beyond test sizes; the
fold reads that part as the single kernel does.  Reference rule:
accumulators.py:86-195 (cumulative / window), providers.py:205-210.
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


def _oracle_pixel_screen_geometric(inst):
    edges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    r = next(iter(inst.coords.values())).shape[0]
    return np.stack([ora.geometric_screen_index(inst.coords, edges, k) for k in range(r)])


@pytest.mark.parametrize('strategy', ['split', 'paged'])
def test_split_finalize_matches_oracle_across_state_changes(strategy, knobs):
    knobs(LDE_FIN_SPLIT=1)  # an exact variant (diagnostics build), off by default
    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()  # T = 100: the split finalize applies
    lo, hi = 10, 90
    eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                        n_screen=view.n_screen, strategy=strategy, toa_range=(lo, hi))
    ps = _oracle_pixel_screen_geometric(inst)
    S, T = view.n_screen, len(edges) - 1

    def fresh_oracle():
        return ora.OracleDetectorView(detector_number=inst.detector_number, pixel_screen=ps,
                                      screen_shape=(80, 320), toa_edges_ns=edges,
                                      toa_slice=(lo, hi))

    o = fresh_oracle()
    n_acc = 0  # the oracle cycles the replicas per accumulate from its start
    # (images only | with histograms | reset before) per step
    plan = ['img', 'img', 'hist', 'img', 'img', 'reset', 'img', 'img']
    for step, what in enumerate(plan):
        if what == 'reset':
            eng.reset_cumulative()
            o, n_acc = fresh_oracle(), 0
            continue
        pid, toa = synthetic.dream_events(400_000, inst, seed=500 + step)
        pid[:100] = 229376  # unknown id
        eng.stage(pid, toa)
        eng.accumulate(n_acc % view.n_replicas)
        n_acc += 1
        o.accumulate(pid, toa)
        res = eng.finalize(images=True, hists=what == 'hist')
        exp = o.finalize()
        np.testing.assert_array_equal(res.current_image.reshape(80, 320), exp['current'],
                                      err_msg=f'step {step}')
        np.testing.assert_array_equal(res.cumulative_image.reshape(80, 320), exp['cumulative'])
        assert res.current_total == exp['counts_total']
        assert res.cumulative_total == exp['counts_total_cumulative']
        assert res.current_in_range == exp['counts_in_toa_range']
        assert res.cumulative_in_range == exp['counts_in_toa_range_cumulative']
        if what == 'hist':
            np.testing.assert_array_equal(res.cumulative_hist, exp['histogram_cumulative'])
        # the fold ran behind the outputs: the cumulative histogram is complete
        # when read (stream order); the window has no data until the next batch
        np.testing.assert_array_equal(eng.read_histogram('cumulative').reshape(S, T),
                                      exp['histogram_cumulative'])
        with pytest.raises(ValueError, match='No data'):
            eng.read_histogram('current')


def test_split_finalize_off_matches_on(knobs):
    """The single-kernel finalize (the default) and the split one
    (LDE_FIN_SPLIT=1, diagnostics build) publish the same images and totals."""
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    edges = inst.edges.edges_ns()
    outs = []
    for split in ('1', '0'):
        knobs(LDE_FIN_SPLIT=split)
        from esslivedata_amd.engine import BinningEngine

        eng = BinningEngine(toa_edges_ns=edges, out_lut=view.lut, pid_offset=view.pid_offset,
                            n_screen=view.n_screen, toa_range=(5, 60))
        got = []
        for step in range(3):
            pid, toa = synthetic.dream_events(300_000, inst, seed=900 + step)
            eng.stage(pid, toa)
            eng.accumulate(step)
            r = eng.finalize(images=True)
            got.append((r.current_image.copy(), r.cumulative_image.copy(), r.current_total,
                        r.current_in_range, r.cumulative_total, r.cumulative_in_range))
        eng.close()
        outs.append(got)
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        assert a[2:] == b[2:]
