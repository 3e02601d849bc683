import os
import sys

import pytest

# the library's fault-injection hooks (CASIM_PLAN_FAIL_ROUND, CASIM_PLAN_WINDOW, ...) are
# read only with CASIM_TEST_HOOKS set (casim_internal.h test_hook_env)
os.environ.setdefault("CASIM_TEST_HOOKS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libcasim.so")


@pytest.fixture(scope="session")
def oracle_lib():
    import pyoracle
    pyoracle.build()
    return pyoracle


def gpu_available() -> bool:
    try:
        from autoscaler_amd import native
        return native.device_count() > 0
    except Exception:
        return False
