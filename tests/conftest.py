import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def digits(a, b):
    """testreport's 'digits of similarity' (verification/testreport:956-986):
    -log10(|a-b| / avg(|a|,|b|)); 16 when identical."""
    import math
    if a == b:
        return 16.0
    avg = 0.5 * (abs(a) + abs(b))
    if avg == 0.0:
        return 16.0
    return -math.log10(abs(a - b) / avg)


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
