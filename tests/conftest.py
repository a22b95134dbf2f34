import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def load_golden(name):
    import json
    path = os.path.join(ROOT, "tests", "golden", name)
    with open(path, encoding="utf-8") as f:
        if name.endswith(".jsonl"):
            return [json.loads(line) for line in f if line.strip()]
        return json.load(f)


@pytest.fixture(scope="session")
def golden_tables():
    return load_golden("tables.json")


@pytest.fixture(scope="session")
def golden_interp():
    return load_golden("interp_py.jsonl")
