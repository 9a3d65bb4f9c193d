"""Host choice of the SIEVE hot rows' TOA window (csrc/lde_window.h), on the
CPU through a small g++-built probe: on DREAM's skewed stream (events
concentrated in the upper geometric TOA bins) it narrows the rows and so
raises the estimated hot fraction; on flat TOA it keeps whole rows."""

import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope='module')
def probe(tmp_path_factory):
    so = tmp_path_factory.mktemp('window') / 'window_probe.so'
    subprocess.run(['g++', '-O2', '-std=c++17', '-shared', '-fPIC', str(HERE / 'native' / 'window_probe.cpp'),
                    '-o', str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.probe_window.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]

    def call(screen_cnt, toa_hist, whole_rows, row_words):
        sc = np.ascontiguousarray(screen_cnt, dtype=np.uint32)
        th = np.ascontiguousarray(toa_hist, dtype=np.uint32)
        out = np.zeros(3, dtype=np.int32)
        est = np.zeros(2, dtype=np.float64)
        lib.probe_window(sc.ctypes.data, sc.size, th.ctypes.data, th.size, whole_rows, row_words,
                         out.ctypes.data, est.ctypes.data)
        return tuple(int(x) for x in out), tuple(est)

    return call


def _dream_sample(n=400_000):
    from esslivedata_amd import projection, synthetic

    inst = synthetic.dream_mantle()
    e = inst.edges.edges_ns()
    pid, toa = synthetic.dream_events(n, inst, seed=7)
    view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution)
    T = len(e) - 1
    b = np.searchsorted(e, toa, side='right') - 1
    scr = view.lut[0][pid - view.pid_offset]
    sc = np.bincount(scr[scr >= 0], minlength=view.n_screen)
    th = np.bincount(b[(b >= 0) & (b < T)], minlength=T)
    return sc, th, T


def test_dream_rows_narrow_to_the_busy_bins(probe):
    sc, th, T = _dream_sample()
    whole = 232
    (rows, w, lo), (win, est) = probe(sc, th, whole, whole * T)
    share_whole = np.sort(sc)[::-1][:whole].sum() / sc.sum()
    assert w < T and rows > whole
    assert win >= 0.99  # the window keeps almost every event of a hot screen
    assert est > share_whole + 0.02  # several points more events hot
    # the window holds the busiest bins: none outside it is busier than one inside
    inside = th[lo:lo + w]
    assert th[:lo].max(initial=0) <= inside.min() and th[lo + w:].max(initial=0) <= inside.min()


def test_flat_toa_keeps_whole_rows(probe):
    sc, _, T = _dream_sample(100_000)
    (rows, w, lo), _ = probe(sc, np.full(T, 1000), 232, 232 * T)
    assert (rows, w, lo) == (232, T, 0)


def test_empty_sample_keeps_whole_rows(probe):
    (rows, w, lo), _ = probe(np.zeros(50), np.zeros(100), 20, 2000)
    assert (rows, w, lo) == (20, 100, 0)
