"""ctypes wrapper of oracle/binning_ref.c (TEST INFRASTRUCTURE / CPU baseline).

Only tests/, smoke() and bench.py's cpu_baseline leg use this module.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = HERE / 'binning_ref.c'
LIB = HERE / 'libbinning_ref.so'


def build(force: bool = False) -> Path:
    if force or not LIB.exists() or LIB.stat().st_mtime < SRC.stat().st_mtime:
        tmp = LIB.with_suffix('.so.tmp')
        subprocess.run(
            ['gcc', '-O3', '-march=x86-64-v2', '-fopenmp', '-fPIC', '-shared', str(SRC), '-o', str(tmp)],
            check=True,
        )
        os.replace(tmp, LIB)
    return LIB


def _lib():
    lib = ctypes.CDLL(str(build()))
    P = ctypes.c_void_p
    lib.ref_bin_batch.restype = ctypes.c_int
    lib.ref_bin_batch.argtypes = [P, P, ctypes.c_int64, P, ctypes.c_int32, ctypes.c_int64, P,
                                  ctypes.c_int64, P, ctypes.c_int64, P, ctypes.c_int]
    return lib


class CDetectorView:
    """Per-batch group -> project -> hist -> += in C with OpenMP threads."""

    def __init__(self, detector_number, pixel_screen, n_screen, toa_edges_ns, threads=0):
        dn = np.asarray(detector_number).ravel().astype(np.int64)
        self.pid_offset = int(dn.min())
        self.pid_table = np.full(int(dn.max()) - self.pid_offset + 1, -1, dtype=np.int64)
        self.pid_table[dn - self.pid_offset] = np.arange(dn.size)
        self.pixel_screen = np.ascontiguousarray(np.atleast_2d(pixel_screen), dtype=np.int64)
        self.S = int(n_screen)
        self.edges = np.ascontiguousarray(toa_edges_ns, dtype=np.float64)
        self.T = len(self.edges) - 1
        self.threads = threads
        self.hist = np.zeros(self.S * self.T, dtype=np.uint64)
        self.threads_used = 1
        self._lib = _lib()

    def accumulate(self, pid, toa, replica=0):
        pid = np.ascontiguousarray(pid, dtype=np.int32)
        toa = np.ascontiguousarray(toa, dtype=np.int32)
        ps = self.pixel_screen[replica]
        self.threads_used = self._lib.ref_bin_batch(
            pid.ctypes.data, toa.ctypes.data, len(pid), self.pid_table.ctypes.data,
            self.pid_offset, len(self.pid_table), ps.ctypes.data, self.S,
            self.edges.ctypes.data, self.T, self.hist.ctypes.data, self.threads)
        return self.hist
