"""Per-test parity numbers (flipped paths, relative errors) collected while the tests run and
written in the terminal summary by tests/conftest.py, so a `pytest -q` log shows them for passing
tests too (their prints are captured)."""
import os

RECORDS = []


def report(**numbers):
    """Record this test's numbers under its node id (PYTEST_CURRENT_TEST)."""
    name = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    RECORDS.append((name, numbers))
