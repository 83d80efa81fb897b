import os
import sys

import pytest

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
    from bitcaskdb_amd import Context, _lib
    c = Context(0)
    if os.environ.get("BCW_TEST_DECODE_PATH"):  # bring-up: pin the default context's decode path
        c.set_option(_lib.OPT_DECODE_PATH, int(os.environ["BCW_TEST_DECODE_PATH"]))
    yield c
    c.close()


@pytest.fixture(scope="session")
def ctx_two():
    """a context pinned to the two-launch decode (k_chase + k_crc; BCW_OPT_DECODE_PATH 1)"""
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from bitcaskdb_amd import Context, _lib
    c = Context(0)
    c.set_option(_lib.OPT_DECODE_PATH, 1)
    c.set_option(_lib.OPT_DECODE_CHUNKS, 1)
    yield c
    c.close()


@pytest.fixture(scope="session")
def ctx_chunks():
    """the two-launch decode over two chunks from 128 blocks on (BCW_OPT_DECODE_CHUNKS 3)"""
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from bitcaskdb_amd import Context, _lib
    c = Context(0)
    c.set_option(_lib.OPT_DECODE_PATH, 1)
    c.set_option(_lib.OPT_DECODE_CHUNKS, 3)
    yield c
    c.close()


@pytest.fixture(scope="session")
def ctx_scan():
    """a context pinned to the one-launch decode (k_scan; BCW_OPT_DECODE_PATH 0)"""
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from bitcaskdb_amd import Context, _lib
    c = Context(0)
    c.set_option(_lib.OPT_DECODE_PATH, 0)
    yield c
    c.close()


@pytest.fixture(params=["scan", "two", "chunks"])
def ctx_path(request, ctx_scan, ctx_two, ctx_chunks):
    """both decode paths: the one-launch k_scan, and k_chase + k_crc over one chunk and over two"""
    return {"scan": ctx_scan, "two": ctx_two, "chunks": ctx_chunks}[request.param]
