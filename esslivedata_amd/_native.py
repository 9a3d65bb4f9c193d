"""ctypes binding of the C ABI in ``include/lde.h``.

The product path has exactly one implementation: the HIP engine in
``libesslivedata_amd.so``.  If the library is missing or cannot be loaded the
import of :func:`lib` raises -- there is no CPU fallback.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / 'libesslivedata_amd.so'
# the diagnostics build (python -m esslivedata_amd.build --diagnostics)
DIAG_LIB_PATH = Path(__file__).resolve().parent / 'libesslivedata_amd_diag.so'
if os.environ.get('LDE_LIBRARY'):  # A/B diagnostics: another build of the same ABI
    LIB_PATH = Path(os.environ['LDE_LIBRARY']).resolve()
    import sys

    print(f'esslivedata_amd: LDE_LIBRARY set, loading {LIB_PATH} instead of the product '
          f'library', file=sys.stderr)

ABI_VERSION = 1

LDE_OK = 0
LDE_EINVAL = -1
LDE_ESTATE = -2
LDE_ENOMEM = -3
LDE_EHIP = -4
LDE_ENODATA = -5
LDE_ENOTSUP = -6

LDE_F64 = 0
LDE_F32 = 1

STRATEGIES = {'auto': 0, 'atomic': 1, 'partition': 2, 'paged': 3, 'split': 4, 'pixel': 5, 'wide': 6}

LDE_CURRENT = 0
LDE_CUMULATIVE = 1

COUNTERS = {
    'pix_overflow': 0,
    'pix_overflow_cap': 1,
    'pix_predicted': 2,
    'waits': 3,
    'waits_blocked': 4,
    'wait_pred_us': 5,
    # 6, 7: reserved (removed sieve counters, read as 0)
    'wide_levels': 8,
    'wide_parts': 9,
    'wide_tree_words': 10,
    'wide_tree_lds': 11,
    'wide_items': 12,
}

KERNELS = {
    'atomic': 0,
    'partition': 1,
    'plan': 2,
    'tile_accumulate': 3,
    'monitor': 4,
    'finalize': 5,
    'binning': 6,
    'paged': 7,
    'page_plan': 8,
    'page_accumulate': 9,
    'split': 10,
    'split_aux': 11,
    'coord': 12,
    'pixel': 13,
    'wide': 14,
    'wide_accumulate': 15,
}

# every symbol include/lde.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    'lde_abi_version',
    'lde_last_error',
    'lde_create',
    'lde_destroy',
    'lde_stage',
    'lde_stage_device',
    'lde_stage_device_batch',
    'lde_ev44_decode',
    'lde_stage_ev44',
    'lde_rebin_f64',
    'lde_accumulate',
    'lde_finalize',
    'lde_finalize_begin',
    'lde_finalize_end',
    'lde_read_histogram',
    'lde_clear',
    'lde_reset_cumulative',
    'lde_export_window',
    'lde_finalize_partials',
    'lde_accumulate_push',
    'lde_push_u64',
    'lde_import_window',
    'lde_export_window_u64',
    'lde_import_window_u64',
    'lde_get_stream',
    'lde_set_lut',
    'lde_set_coord_lut',
    'lde_synchronize',
    'lde_timing_enable',
    'lde_timing_select',
    'lde_kernel_stats',
    'lde_info',
    'lde_counter',
    'lde_set_groups',
    'lde_group_spectra',
    'lde_host_alloc',
    'lde_host_free',
)

MAX_GROUP_SETS = 4


class LdeConfig(ctypes.Structure):
    _fields_ = [
        ('abi_version', ctypes.c_int32),
        ('device_id', ctypes.c_int32),
        ('stream', ctypes.c_void_p),
        ('pid_offset', ctypes.c_int32),
        ('n_replicas', ctypes.c_int32),
        ('lut_len', ctypes.c_int64),
        ('out_lut', ctypes.POINTER(ctypes.c_int32)),
        ('n_screen', ctypes.c_int64),
        ('n_toa_bins', ctypes.c_int32),
        ('toa_edges', ctypes.POINTER(ctypes.c_double)),
        ('out_dtype', ctypes.c_int32),
        ('strategy', ctypes.c_int32),
        ('range_lo', ctypes.c_int32),
        ('range_hi', ctypes.c_int32),
    ]


class LdeCoordLut(ctypes.Structure):
    _fields_ = [
        ('pixel_distance', ctypes.c_void_p),
        ('n_pixels', ctypes.c_int64),
        ('table', ctypes.c_void_p),
        ('n_dist', ctypes.c_int32),
        ('n_time', ctypes.c_int32),
        ('dist0', ctypes.c_double),
        ('dist_step', ctypes.c_double),
        ('time0', ctypes.c_double),
        ('time_step', ctypes.c_double),
    ]


class LdeOutputs(ctypes.Structure):
    _fields_ = [
        ('current_image', ctypes.c_void_p),
        ('cumulative_image', ctypes.c_void_p),
        ('current_hist', ctypes.c_void_p),
        ('cumulative_hist', ctypes.c_void_p),
        ('totals', ctypes.c_uint64 * 4),
    ]


_lock = threading.Lock()
_libs: dict[bool, ctypes.CDLL] = {}
# engines created while this is set load the diagnostics build (tests only:
# the parity matrix over the engine's tuning variants, diagnostics_library())
_use_diag = False


def _declare(lib: ctypes.CDLL) -> None:
    H = ctypes.c_void_p
    i32, i64 = ctypes.c_int32, ctypes.c_int64
    P = ctypes.c_void_p
    sig = {
        'lde_abi_version': (ctypes.c_int, []),
        'lde_last_error': (ctypes.c_char_p, [H]),
        'lde_create': (ctypes.c_int, [ctypes.POINTER(LdeConfig), ctypes.POINTER(H)]),
        'lde_destroy': (None, [H]),
        'lde_stage': (ctypes.c_int, [H, P, P, i64]),
        'lde_stage_device': (ctypes.c_int, [H, P, P, i64]),
        'lde_stage_device_batch': (ctypes.c_int, [H, i64, P, P, P]),
        'lde_ev44_decode': (ctypes.c_int, [P, i64, P]),
        'lde_rebin_f64': (ctypes.c_int, [P, P, i64, P, i64, P, P, P]),
        'lde_stage_ev44': (ctypes.c_int, [H, P, i64, i64, i32, ctypes.POINTER(i64)]),
        'lde_accumulate': (ctypes.c_int, [H, i32]),
        'lde_finalize': (ctypes.c_int, [H, ctypes.POINTER(LdeOutputs)]),
        'lde_finalize_begin': (ctypes.c_int, [H, ctypes.POINTER(LdeOutputs)]),
        'lde_finalize_end': (ctypes.c_int, [H, ctypes.POINTER(LdeOutputs)]),
        'lde_read_histogram': (ctypes.c_int, [H, i32, P]),
        'lde_clear': (ctypes.c_int, [H]),
        'lde_reset_cumulative': (ctypes.c_int, [H]),
        'lde_export_window': (ctypes.c_int, [H, P]),
        'lde_finalize_partials': (ctypes.c_int, [H, P]),
        'lde_accumulate_push': (ctypes.c_int, [H, i32, P]),
        'lde_push_u64': (ctypes.c_int, [H, P]),
        'lde_import_window': (ctypes.c_int, [H, P]),
        'lde_export_window_u64': (ctypes.c_int, [H, P]),
        'lde_import_window_u64': (ctypes.c_int, [H, P]),
        'lde_get_stream': (ctypes.c_int, [H, ctypes.POINTER(ctypes.c_void_p)]),
        'lde_set_lut': (ctypes.c_int, [H, P]),
        'lde_set_coord_lut': (ctypes.c_int, [H, ctypes.POINTER(LdeCoordLut)]),
        'lde_synchronize': (ctypes.c_int, [H]),
        'lde_set_groups': (ctypes.c_int, [H, i32, i64, P, P]),
        'lde_group_spectra': (ctypes.c_int, [H, i32, i32, P]),
        'lde_host_alloc': (ctypes.c_int, [i64, ctypes.POINTER(ctypes.c_void_p)]),
        'lde_host_free': (ctypes.c_int, [P]),
        'lde_timing_enable': (ctypes.c_int, [H, i32]),
        'lde_timing_select': (ctypes.c_int, [H, ctypes.c_uint32]),
        'lde_kernel_stats': (
            ctypes.c_int,
            [H, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64)],
        ),
        'lde_counter': (ctypes.c_int, [H, i32, ctypes.POINTER(i64)]),
        'lde_info': (
            ctypes.c_int,
            [
                H,
                ctypes.POINTER(i64),
                ctypes.POINTER(i32),
                ctypes.POINTER(i64),
                ctypes.POINTER(i32),
                ctypes.POINTER(i32),
                ctypes.POINTER(i64),
                ctypes.POINTER(i32),
            ],
        ),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib(diagnostics: bool | None = None) -> ctypes.CDLL:
    """Load the engine library (once).  Raises if it is missing.
    ``diagnostics`` (default: inside :func:`diagnostics_library`) loads the
    diagnostics build instead, whose tuning knobs (``LDE_*`` variables) select
    the engine's internal kernel variants; the product library fixes them."""
    diag = _use_diag if diagnostics is None else bool(diagnostics)
    with _lock:
        if diag in _libs:
            return _libs[diag]
        path = DIAG_LIB_PATH if diag else LIB_PATH
        if not path.exists():
            raise RuntimeError(
                f'HIP engine library {path} is missing; build it with '
                f'`python -m esslivedata_amd.build{" --diagnostics" if diag else ""}` '
                '(no CPU fallback exists)'
            )
        try:  # share torch's HIP runtime (same SONAME) when torch is present
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is part of the image
            pass
        # both builds may be loaded side by side (-Bsymbolic: each binds its
        # own symbols); only the product library goes into the global scope
        cdll = ctypes.CDLL(str(path), mode=ctypes.RTLD_LOCAL if diag else ctypes.RTLD_GLOBAL)
        _declare(cdll)
        if cdll.lde_abi_version() != ABI_VERSION:
            raise RuntimeError('libesslivedata_amd ABI version mismatch')
        _libs[diag] = cdll
        return cdll


@contextlib.contextmanager
def diagnostics_library():
    """Engines created inside use the diagnostics build (test infrastructure)."""
    global _use_diag
    prev, _use_diag = _use_diag, True
    try:
        yield lib(True)
    finally:
        _use_diag = prev


def last_error(handle, library: ctypes.CDLL | None = None) -> str:
    msg = (library or lib()).lde_last_error(handle)
    return msg.decode() if msg else ''


def check(rc: int, handle=None, library: ctypes.CDLL | None = None) -> None:
    """Map engine error codes onto the reference's exception conventions
    (``library``: the build the handle belongs to)."""
    if rc == LDE_OK:
        return
    msg = last_error(handle, library)
    if rc in (LDE_EINVAL, LDE_ENODATA):
        raise ValueError(msg)
    if rc == LDE_ENOTSUP:
        raise NotImplementedError(msg)
    raise RuntimeError(msg or f'lde error {rc}')
