import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The tests that force a code path (work splits, slab depths, bin chunk sizes) do so through the
# library's TVAM_* tuning knobs, which it honours only under TVAM_EXPERIMENTAL=1 (tvam_knob, read at
# plan creation): each such test sets both with monkeypatch (the `knobs` fixture); every other test
# runs the production defaults.
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and libtvam.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """The parity numbers the tests recorded (tests/parity_report.py): flipped paths per test."""
    from parity_report import RECORDS
    if not RECORDS:
        return
    terminalreporter.section("parity report (flip protocol: flipped paths, errors outside them)")
    for name, numbers in RECORDS:
        terminalreporter.write_line(f"{name}: " + ", ".join(
            f"{k} {v:.3e}" if isinstance(v, float) else f"{k} {v}" for k, v in numbers.items()))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.build()
    return orc


@pytest.fixture
def knobs(monkeypatch):
    """knobs(NAME=value, ...): set tuning knobs for this test, with TVAM_EXPERIMENTAL=1."""
    def set_(**kv):
        monkeypatch.setenv("TVAM_EXPERIMENTAL", "1")
        for k, v in kv.items():
            monkeypatch.setenv(k, str(v))
    return set_
