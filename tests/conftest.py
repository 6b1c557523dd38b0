import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)
# the tests exercise every kernel family and schedule through the A/B option keys, which the
# library accepts only with IQO_HIP_TUNING set (include/iqo_hip.h iqo_hip_plan_set_option)
os.environ.setdefault("IQO_HIP_TUNING", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(HERE, "golden", "golden.json")) as f:
        return json.load(f)
