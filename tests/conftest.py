import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librtamd.so on cuda:0)")
    config.addinivalue_line("markers", "slow: CPU test taking more than ~10 s")


@pytest.fixture(scope="session")
def workdir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("scenes"))


@pytest.fixture(scope="session")
def gpu_available():
    import raytracert_amd as R
    n = R.device_count()
    if n < 1:
        pytest.fail("no HIP device visible to librtamd.so (gpu-marked test run without a GPU)")
    return n
