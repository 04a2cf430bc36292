import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def corpora():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "corpora.json")) as f:
        return json.load(f)
