import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device) to run')
    config.addinivalue_line('markers', 'slow: long-running test')


@pytest.fixture(scope='session')
def engine_lib():
    """The built HIP engine library (build it if missing; also the diagnostics
    build the ``knobs`` fixture loads)."""
    from esslivedata_amd import build

    build.build()
    build.build(diagnostics=True)
    from esslivedata_amd import _native

    return _native.lib()


@pytest.fixture
def knobs(monkeypatch, engine_lib):
    """Engine tuning knobs for one test: ``knobs(LDE_X=v, ...)`` sets the
    variables, and every engine the test creates loads the diagnostics build,
    the only one that reads them (the product library fixes its tuning)."""
    from esslivedata_amd import _native

    cm = _native.diagnostics_library()
    cm.__enter__()

    def set_(**kv):
        for k, v in kv.items():
            monkeypatch.setenv(k, str(v))

    try:
        yield set_
    finally:
        cm.__exit__(None, None, None)
