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
ARCH = os.environ.get('LDE_OFFLOAD_ARCH', 'gfx950')


def _hipcc() -> str:
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if cand and (os.path.sep not in cand or Path(cand).exists()):
            return cand
    raise RuntimeError('hipcc not found')


def sources() -> list[Path]:
    return sorted(CSRC.glob('*.hip')) + sorted(CSRC.glob('*.cpp'))


def needs_build() -> bool:
    if not LIB.exists():
        return True
    mtime = LIB.stat().st_mtime
    deps = sources() + sorted(CSRC.glob('*.h')) + [ROOT / 'include' / 'lde.h']
    return any(p.stat().st_mtime > mtime for p in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB
    tmp = LIB.with_suffix('.so.tmp')
    cmd = [
        _hipcc(),
        f'--offload-arch={ARCH}',
        '-O3',
        '-std=c++17',
        '-fPIC',
        '-shared',
        '-Wall',
        '-Wno-unused-function',
        '-Wno-unused-result',
        f'-I{ROOT / "include"}',
        *[str(s) for s in sources()],
        '-o',
        str(tmp),
    ]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}')
    if verbose and res.stderr.strip():
        print(res.stderr, file=sys.stderr)
    os.replace(tmp, LIB)
    return LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
