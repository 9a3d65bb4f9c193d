"""Build the in-tree HIP engine library for gfx950 (MI355X).

``python -m esslivedata_amd.build`` compiles ``csrc/*.hip`` + ``csrc/*.cpp``
into ``esslivedata_amd/libesslivedata_amd.so`` with hipcc.  The library is
git-ignored but travels with the working tree to the GPU box.
"""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / 'csrc'
LIB = PKG / 'libesslivedata_amd.so'
# -DLDE_DIAGNOSTICS: adds the timing ablations (wrong results by design) the
# product library refuses; loaded only through LDE_LIBRARY by the A/B tools
DIAG_LIB = PKG / 'libesslivedata_amd_diag.so'
ARCH = os.environ.get('LDE_OFFLOAD_ARCH', 'gfx950')


def _hipcc() -> str:
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if cand and (os.path.sep not in cand or Path(cand).exists()):
            return cand
    raise RuntimeError('hipcc not found')


def sources() -> list[Path]:
    return sorted(CSRC.glob('*.hip')) + sorted(CSRC.glob('*.cpp'))


def needs_build(lib: Path = LIB) -> bool:
    if not lib.exists():
        return True
    mtime = lib.stat().st_mtime
    deps = sources() + sorted(CSRC.glob('*.h')) + [ROOT / 'include' / 'lde.h']
    return any(p.stat().st_mtime > mtime for p in deps)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}')
    if verbose and res.stderr.strip():
        print(res.stderr, file=sys.stderr)


def build(force: bool = False, verbose: bool = False, diagnostics: bool = False) -> Path:
    """Compile every source to an object in parallel, then link the library
    (the product library; ``diagnostics=True`` the separate diagnostics one)."""
    lib = DIAG_LIB if diagnostics else LIB
    if not force and not needs_build(lib):
        return lib
    from concurrent.futures import ThreadPoolExecutor

    flags = [
        f'--offload-arch={ARCH}',
        '-O3',
        '-std=c++17',
        '-fPIC',
        '-Wall',
        '-Wno-unused-function',
        '-Wno-unused-result',
        f'-I{ROOT / "include"}',
    ]
    if diagnostics:
        flags.append('-DLDE_DIAGNOSTICS')
    objdir = PKG / ('build_diag' if diagnostics else 'build')
    objdir.mkdir(exist_ok=True)
    srcs = sources()
    objs = [objdir / (s.name + '.o') for s in srcs]
    jobs = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_run, [_hipcc(), *flags, '-c', str(s), '-o', str(o)], verbose)
                for s, o in zip(srcs, objs)]
        for f in futs:
            f.result()
    tmp = lib.with_suffix('.so.tmp')
    _run([_hipcc(), f'--offload-arch={ARCH}', '-shared', '-fPIC', '-Wl,--no-undefined', '-Wl,-Bsymbolic',
          *[str(o) for o in objs], '-o',
          str(tmp)], verbose)
    os.replace(tmp, lib)
    return lib


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True,
                diagnostics='--diagnostics' in sys.argv))
