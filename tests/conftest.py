import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the tests that force a code path (work splits, slab depths, bin chunk sizes) do so through the
# library's TVAM_* tuning knobs, which it honours only under TVAM_EXPERIMENTAL=1 (tvam_knob)
os.environ.setdefault("TVAM_EXPERIMENTAL", "1")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and libtvam.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.build()
    return orc
