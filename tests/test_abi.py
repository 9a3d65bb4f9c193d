"""The C-ABI library loads and exports every symbol include/lde.h declares.

CPU only: no compute call is made (no GPU in the build container).
"""

import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / 'include' / 'lde.h').read_text()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char \*)\s*\**(lde_\w+)\s*\(', text, re.M)))


def test_header_declarations_match_binding(engine_lib):
    from esslivedata_amd import _native

    assert declared_symbols() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(engine_lib):
    for name in declared_symbols():
        assert hasattr(engine_lib, name), name
    assert engine_lib.lde_abi_version() == 1


def test_create_rejects_bad_config_without_device(engine_lib):
    from esslivedata_amd import _native

    h = ctypes.c_void_p()
    assert engine_lib.lde_create(None, ctypes.byref(h)) == _native.LDE_EINVAL
    assert b'config is NULL' in engine_lib.lde_last_error(None)
    cfg = _native.LdeConfig()
    cfg.abi_version = 99
    assert engine_lib.lde_create(ctypes.byref(cfg), ctypes.byref(h)) == _native.LDE_EINVAL
    assert b'abi_version' in engine_lib.lde_last_error(None)
    assert not h.value
    with pytest.raises(ValueError):
        _native.check(_native.LDE_EINVAL)
    with pytest.raises(RuntimeError):
        _native.check(_native.LDE_EHIP)


def test_null_handle_calls_are_rejected(engine_lib):
    from esslivedata_amd import _native

    assert engine_lib.lde_accumulate(None, 0) == _native.LDE_EINVAL
    assert engine_lib.lde_finalize(None, None) == _native.LDE_EINVAL
    assert engine_lib.lde_stage(None, None, None, 0) == _native.LDE_EINVAL
    engine_lib.lde_destroy(None)  # no-op


def test_library_is_gfx950_code_object():
    import subprocess

    lib = ROOT / 'esslivedata_amd' / 'libesslivedata_amd.so'
    out = subprocess.run(
        ['/opt/rocm/lib/llvm/bin/llvm-readelf', '-S', str(lib)], capture_output=True, text=True
    ).stdout
    assert '.hip_fatbin' in out
    blob = lib.read_bytes()
    assert b'gfx950' in blob


@pytest.mark.parametrize('knob', ['LDE_SIEVE_ABLATE', 'LDE_ABLATE', 'LDE_COLD_SORT_ABLATE'])
def test_product_library_refuses_diagnostic_ablations(knob):
    """Result-corrupting timing ablations exist only in the LDE_DIAGNOSTICS
    build: the product library's lde_create refuses them (before any device
    call, so this runs without a GPU)."""
    import os
    import subprocess
    import sys

    code = (
        'import ctypes\n'
        'from esslivedata_amd import _native\n'
        'lib = _native.lib()\n'
        'cfg = _native.LdeConfig(); cfg.abi_version = _native.ABI_VERSION\n'
        'h = ctypes.c_void_p()\n'
        'rc = lib.lde_create(ctypes.byref(cfg), ctypes.byref(h))\n'
        'print(rc, lib.lde_last_error(None).decode())\n'
    )
    env = dict(os.environ, **{knob: '1'})
    env.pop('LDE_LIBRARY', None)
    res = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True,
                         cwd=ROOT, timeout=120)
    assert res.returncode == 0, res.stderr
    rc, msg = res.stdout.strip().split(' ', 1)
    assert int(rc) == -1 and knob in msg and 'DIAGNOSTICS' in msg


def test_product_library_has_only_exact_sieve_variants():
    import subprocess

    lib = ROOT / 'esslivedata_amd' / 'libesslivedata_amd.so'
    out = subprocess.run(['nm', '-C', str(lib)], capture_output=True, text=True).stdout
    modes = {int(m) for m in re.findall(r'lde::k_sieve<(\d+), \d>\(', out)}
    # the product build has the plain sieve and the keyed wavelength pass
    # (262144) only: no ablation modes
    assert modes == {0, 262144}, modes
