"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py

Three kinds of fixtures (see DESIGN.md "Parity"):

1. ``reference_kats.json`` -- known answers transcribed from the reference's own
   tests (inputs and expected outputs as data; file:line cited per case).  The
   reference cannot be imported here (Python 3.10 vs >=3.12, scipp/essreduce
   absent), so these literals are the reference's pinned behaviour.
2. ``tie_kats.json`` -- hand-derived edge-tie cases: integer TOAs exactly on,
   below and above float64 edges produced by ``linspace``/``geomspace`` in ms and
   converted to ns with one f64 multiply.  Expected bins were worked out by
   hand from the f64 values printed next to them (e.g. 5.0001 ms * 1e6 =
   5000100.000000001 ns, so TOA 5000100 ns is in bin 6, not 7).
3. ``dream_small.npz`` -- a restatement-generated regression vector (DREAM
   mantle shape, skewed pixels, geomspace edges; 200k events, replica 1) with
   the oracle's histogram, used to pin the GPU engine and to catch oracle drift.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

REFERENCE_KATS = [
    {
        'name': 'group_by_pixel_sizes',
        'source': 'tests/preprocessors/group_by_pixel_test.py:24-45',
        'detector_number': [1, 2, 3],
        'messages': [{'pixel_id': [1, 2, 3, 1, 3], 'toa': [100, 200, 300, 400, 500]}],
        'expected_sizes': [2, 1, 2],
    },
    {
        'name': 'group_by_pixel_two_messages',
        'source': 'tests/preprocessors/group_by_pixel_test.py:47-63',
        'detector_number': [1, 2],
        'messages': [
            {'pixel_id': [1, 2], 'toa': [100, 200]},
            {'pixel_id': [1, 1], 'toa': [300, 400]},
        ],
        'expected_sizes': [3, 1],
    },
    {
        'name': 'group_by_pixel_after_get',
        'source': 'tests/preprocessors/group_by_pixel_test.py:81-93',
        'detector_number': [1, 2],
        'messages': [{'pixel_id': [2], 'toa': [200]}],
        'expected_sizes': [0, 1],
    },
    {
        'name': 'monitor_event_histogram',
        'source': 'tests/workflows/monitor_workflow_test.py:161-183',
        'toa_ns': [1, 2, 3, 4, 5],
        'edges_ns': [0.0, 2.0, 4.0, 6.0, 8.0, 10.0],
        'expected_sum': 5,
        'expected_hist': [1, 2, 2, 0, 0],
    },
    {
        'name': 'monitor_counts_in_range',
        'source': 'tests/workflows/monitor_workflow_test.py:232-243',
        'edges_ns': [0.0, 2.0, 4.0, 6.0, 8.0, 10.0],
        'hist': [1.0, 2.0, 3.0, 4.0, 5.0],
        'range_ns': [2.0, 8.0],
        'expected': 9.0,
    },
    {
        'name': 'monitor_counts_total',
        'source': 'tests/workflows/monitor_workflow_test.py:222-230',
        'hist': [1.0, 2.0, 3.0],
        'expected': 6.0,
    },
    {
        'name': 'detector_service_cumulative_current',
        'source': 'tests/services/detector_data_test.py:57-131',
        'note': 'uniform(0, 70e6) ns TOA (tests/helpers/livedata_app.py:189) is inside the '
        'default 0..71.43 ms edges, so every event with a known pixel id is counted',
        'batches': [[2000], [3000], [1000, 1000]],
        'expected_cumulative': [2000, 5000, 7000],
        'expected_current': [2000, 3000, 2000],
    },
]



def _fake_nexus_events(y_size: int, x_size: int, n_per_pixel: int) -> dict:
    """Inputs of tests/workflows/detector_view/utils.py:13-60
    (make_fake_nexus_detector_data): event ids repeat(arange(1, P + 1), n),
    event_time_offset = default_rng(42).uniform(0, 71e6) ns.  numpy's
    generator, so the values are the reference test's own; the engine's wire
    type is int32 ns, so the TOAs are stored floored (all stay in 0..71 ms)."""
    rng = np.random.default_rng(42)
    p = y_size * x_size
    eto = rng.uniform(0, 71_000_000, p * n_per_pixel)
    return {'event_id': np.repeat(np.arange(1, p + 1), n_per_pixel).tolist(),
            'toa': np.floor(eto).astype(np.int64).tolist()}


def _screen_coords(n_pixels: int, screen_shape: tuple[int, int]) -> dict:
    """projectors_test.py:19-54 (make_screen_coords_and_edges): two replicas,
    x = pixel_x * scale + noise, y = pixel_y * scale + noise with the same
    default_rng(42).normal(0, 0.1) noise for x and y of a replica."""
    n_replicas = 2
    det_side = int(np.sqrt(n_pixels))
    scale_x = screen_shape[0] / det_side
    scale_y = screen_shape[1] / det_side
    pixel_y = np.arange(n_pixels) // det_side
    pixel_x = np.arange(n_pixels) % det_side
    rng = np.random.default_rng(42)
    xs, ys = [], []
    for _ in range(n_replicas):
        noise = rng.normal(0, 0.1, n_pixels)
        xs.append((pixel_x * scale_x + noise).tolist())
        ys.append((pixel_y * scale_y + noise).tolist())
    return {'screen_x': xs, 'screen_y': ys}


def _windows_multiple_pushes() -> list[int]:
    """accumulators_test.py:360-389: the number of pushes of each of the 10
    windows, drawn with the test's own RNG consumption order
    (default_rng(123): integers(1, 5) per window, random() per push)."""
    rng = np.random.default_rng(seed=123)
    out = []
    for _ in range(10):
        n = int(rng.integers(1, 5))
        for _ in range(n):
            rng.random()
        out.append(n)
    return out


def reference_kats_r2() -> list[dict]:
    ev44 = _fake_nexus_events(4, 4, 10)
    flip_ev = _fake_nexus_events(2, 3, 50)
    n_push = _windows_multiple_pushes()
    win_exp, cum = [], [0, 0]
    for n in n_push:
        w = [sum(range(n)), sum(range(1, n + 1))]
        win_exp.append(w)
        cum = [cum[0] + w[0], cum[1] + w[1]]
    return [
        {
            'name': 'projector_count_conservation',
            'source': 'tests/workflows/detector_view/projectors_test.py:56-75',
            'detector_number': list(range(1, 17)),
            'events': ev44,
            'coords': _screen_coords(16, (4, 4)),
            'edges': {'screen_x': np.linspace(-1, 5, 10).tolist(),
                      'screen_y': np.linspace(-1, 5, 10).tolist()},
            'replica': 0,
            'expected_total': 160,
        },
        {
            'name': 'projector_replicas_differ',
            'source': 'tests/workflows/detector_view/projectors_test.py:107-121',
            'detector_number': list(range(1, 17)),
            'events': ev44,
            'coords': _screen_coords(16, (4, 4)),
            'edges': {'screen_x': np.linspace(0, 4, 5).tolist(),
                      'screen_y': np.linspace(0, 4, 5).tolist()},
            'expected': 'screen counts of replica 0 and replica 1 differ',
        },
        {
            'name': 'projector_flip_x_mirrors',
            'source': 'tests/workflows/detector_view/projectors_test.py:124-178',
            'detector_number': list(range(1, 7)),
            'events': flip_ev,
            'positions': np.stack([[-0.1, 0.0, 0.1, -0.1, 0.0, 0.1],
                                   [-0.05, -0.05, -0.05, 0.05, 0.05, 0.05],
                                   [2.0] * 6], axis=-1).tolist(),
            'projection_type': 'xy_plane',
            'resolution': {'x': 3, 'y': 2},
            'expected': 'flipped[x=i] == normal[x=n-1-i] for every i; y edges identical',
        },
        {
            'name': 'accumulator_window_accumulates',
            'source': 'tests/preprocessors/accumulators_test.py:260-269',
            'pushes': [[1, 2], [3, 4]],
            'expected_window': [4, 6],
        },
        {
            'name': 'accumulator_window_cleared_on_finalize',
            'source': 'tests/preprocessors/accumulators_test.py:253-258, 271-276',
            'pushes': [[1, 2]],
            'expected': 'window empty after on_finalize; reading it raises ValueError',
        },
        {
            'name': 'accumulator_pair_multiple_cycles',
            'source': 'tests/preprocessors/accumulators_test.py:332-358',
            'cycles': [[i, i + 1] for i in range(20)],
            'expected_cumulative': [sum(range(20)), sum(range(1, 21))],
        },
        {
            'name': 'accumulator_pair_multiple_pushes_per_window',
            'source': 'tests/preprocessors/accumulators_test.py:360-389',
            'note': 'window w receives pushes [j, j + 1] for j < n_pushes[w]',
            'n_pushes': n_push,
            'expected_windows': win_exp,
            'expected_cumulative': cum,
        },
        {
            'name': 'accumulator_reset_on_coord_change',
            'source': 'tests/preprocessors/accumulators_test.py:427-463',
            'cases': [
                {'pushes': [[[1, 2], 0.0], [[3, 4], 0.0]], 'expected_cumulative': [4, 6]},
                {'pushes': [[[1, 2], 0.0], [[3, 4], 1.0]], 'expected_cumulative': [3, 4]},
                {'pushes': [[[1, 2], None], [[3, 4], None]], 'expected_cumulative': [4, 6]},
                {'pushes': [[[1, 2], 0.0], [[3, 4], 1.0]], 'expected_window': [3, 4]},
            ],
        },
        {
            'name': 'monitor_full_workflow_cycle',
            'source': 'tests/workflows/monitor_workflow_test.py:346-391',
            'note': 'event_time_offset [1.5, 2.5, 3.5, 7.5, 8.5] ns in the test; the ev44 '
                    'wire carries int32 ns, so floored here (same bins)',
            'toa_ns': [1, 2, 3, 7, 8],
            'edges_ns': np.linspace(0, 10, 11).tolist(),
            'expected': {'cumulative_sum': 5.0, 'current_sum': 5.0, 'counts_total': 5.0,
                         'counts_in_toa_range': 5.0, 'counts_total_cumulative': 5.0,
                         'counts_in_toa_range_cumulative': 5.0},
        },
    ]


def reference_kats_r5() -> list[dict]:
    """Window time coords (round 5): integer ns scalars as Timestamp.to_scipp()
    makes them (SRC/core/timestamp.py:216-220); the monitor's cumulative
    against its clearing window over two cycles."""
    return [
        {
            'name': 'monitor_cumulative_accumulates_window_clears',
            'source': 'tests/workflows/monitor_workflow_test.py:484-516',
            'note': 'the class fixtures of :349-360: edges linspace(0, 10, 11) ns, '
                    'event_time_offset [1.5, 2.5, 3.5, 7.5, 8.5] ns (floored to int32 ns on '
                    'the ev44 wire: same bins); the same events accumulated in two cycles',
            'toa_ns': [1, 2, 3, 7, 8],
            'edges_ns': np.linspace(0, 10, 11).tolist(),
            'cycles': [[0, 1000], [1000, 2000]],
            'expected': [
                {'cumulative_sum': 5.0, 'current_sum': 5.0},
                {'cumulative_sum': 10.0, 'counts_total_cumulative': 10.0,
                 'counts_in_toa_range_cumulative': 10.0, 'current_sum': 5.0,
                 'counts_total': 5.0, 'counts_in_toa_range': 5.0},
            ],
        },
        {
            'name': 'window_outputs_time_coords',
            'source': 'tests/workflows/detector_view/integration_test.py:28-84',
            'note': '4x4 logical view (fold detector_number 1..16 to y, x), 10 events per '
                    'pixel, ROI rectangle x [0, 2), y [0, 2) (index bounds, unit None)',
            'detector_number': list(range(1, 17)),
            'fold_sizes': {'y': 4, 'x': 4},
            'events': _fake_nexus_events(4, 4, 10),
            'roi_rectangle': {'x': [0, 2], 'y': [0, 2]},
            'start_time_ns': 1000,
            'end_time_ns': 2000,
            'expected': {'start_time': 1000, 'time': 2000, 'unit': 'ns', 'dtype': 'int64'},
            'stamped': ['current', 'counts_total', 'counts_in_toa_range', 'roi_spectra_current'],
            'unstamped': ['cumulative', 'roi_spectra_cumulative', 'counts_total_cumulative',
                          'counts_in_toa_range_cumulative'],
        },
        {
            'name': 'window_time_tracking',
            'source': 'tests/workflows/stream_processor_workflow_test.py:407-516',
            'note': 'each period: accumulate calls [start, end] ns, then finalize (or clear); '
                    'expected (start_time, time) of the window output, null after clear',
            'periods': [
                {'accumulate': [[1000, 2000]], 'then': 'finalize', 'expected': [1000, 2000]},
                {'accumulate': [[1000, 2000], [3000, 4000]], 'then': 'finalize',
                 'expected': [1000, 4000]},
                {'accumulate': [[5000, 6000]], 'then': 'finalize', 'expected': [5000, 6000]},
                {'accumulate': [[7000, 8000]], 'then': 'clear', 'expected': None},
                {'accumulate': [[9000, 10000]], 'then': 'finalize', 'expected': [9000, 10000]},
            ],
        },
    ]


# hand-derived: toa -> expected bin (-1 = dropped)
TIE_KATS = [
    {
        'name': 'default_linear_edges_ms',
        'edges_ms': {'op': 'linspace', 'start': 0.0, 'stop': 71.43, 'num': 101},
        'f64_edges_ns_used': {'1': 714300.0, '7': 5000100.000000001, '10': 7143000.000000001,
                              '100': 71430000.0},
        'cases': [
            [-1, -1], [0, 0], [714299, 0], [714300, 1], [714301, 1],
            [5000099, 6], [5000100, 6], [5000101, 7],
            [7142999, 9], [7143000, 9], [7143001, 10],
            [71429999, 99], [71430000, -1], [71430001, -1],
        ],
    },
    {
        'name': 'geomspace_edges_ms',
        'edges_ms': {'op': 'geomspace', 'start': 0.5, 'stop': 71.43, 'num': 101},
        'f64_edges_ns_used': {'0': 500000.0, '1': 525435.1359694994, '50': 5976202.807803631,
                              '99': 67972233.9734684, '100': 71430000.0},
        'cases': [
            [499999, -1], [500000, 0], [525435, 0], [525436, 1],
            [5976202, 49], [5976203, 50], [67972233, 98], [67972234, 99],
            [71429999, 99], [71430000, -1],
        ],
    },
    {
        'name': 'fractional_and_duplicate_edges_ns',
        'edges_ns': [-5.5, -0.5, 0.0, 0.5, 1.0, 1.0, 2.5, 3.0],
        'cases': [
            [-6, -1], [-5, 0], [-1, 0], [0, 2], [1, 5], [2, 5], [3, -1],
        ],
    },
]

SCREEN_EDGE_KATS = [
    {
        'name': 'int_bin_count_includes_max',
        'note': 'scipp hist({dim: res}) edges = linspace(nanmin, nextafter(nanmax, +inf), res+1)',
        'values': [0.0, 1.0, 2.0, 3.0],
        'res': 2,
        'expected_bins': [0, 0, 1, 1],
    },
    {
        'name': 'nan_dropped',
        'values': [0.0, float('nan'), 4.0],
        'res': 4,
        'expected_bins': [0, -1, 3],
    },
]


def main() -> None:
    # entries transcribed by hand into the JSON (the round-3 logical-view KATs)
    # are kept; the generated ones are replaced in place or appended
    path = HERE / 'reference_kats.json'
    gen = {k['name']: k for k in REFERENCE_KATS + reference_kats_r2() + reference_kats_r5()}
    old = json.loads(path.read_text()) if path.exists() else []
    out = [gen.pop(k['name'], k) for k in old] + list(gen.values())
    path.write_text(json.dumps(out, indent=1))
    (HERE / 'tie_kats.json').write_text(
        json.dumps({'toa': TIE_KATS, 'screen': SCREEN_EDGE_KATS}, indent=1)
    )
    from esslivedata_amd import synthetic
    from oracle import scipp_semantics as ora

    inst = synthetic.dream_mantle()
    edges = {d: ora.screen_edges(inst.coords[d], r) for d, r in inst.resolution.items()}
    pid, toa = synthetic.dream_events(200_000, inst, seed=11)
    pid[:500] = 100  # unknown ids
    ps = ora.geometric_screen_index(inst.coords, edges, 1)
    pix = ora.pixel_index(pid, inst.detector_number)
    hist = ora.detector_histogram(ps, 25600, pix, toa, inst.edges.edges_ns())
    nz = np.nonzero(hist.ravel())[0]
    np.savez_compressed(
        HERE / 'dream_small.npz',
        pid=pid,
        toa=toa,
        replica=np.int32(1),
        hist_index=nz.astype(np.int32),
        hist_value=hist.ravel()[nz].astype(np.int32),
    )
    print('wrote', sorted(p.name for p in HERE.iterdir() if p.suffix in ('.json', '.npz')))


if __name__ == '__main__':
    main()
