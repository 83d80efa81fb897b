import os
import sys

import pytest

# the library's fault-injection option (BCW_OPT_TEST_ABORT_WAIT) is refused unless the process opts in
os.environ.setdefault("BCW_TEST_HOOKS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libbcw.so on the device)")


def gpu_available() -> bool:
    try:
        from bitcaskdb_amd import _lib
        return _lib.lib.bcw_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def ctx():
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from bitcaskdb_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def ctx_path():
    """a context of its own for the decode-path tests (k_chase + k_crc; the one-launch k_scan and the two-chunk
    decode were retired in round 4)"""
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from bitcaskdb_amd import Context
    c = Context(0)
    yield c
    c.close()
