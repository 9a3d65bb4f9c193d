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
    """The built HIP engine library (build it if missing)."""
    from esslivedata_amd import build

    build.build()
    from esslivedata_amd import _native

    return _native.lib()
