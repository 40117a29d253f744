import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def golden():
    from tests.golden_util import load_golden
    return load_golden()


@pytest.fixture(autouse=True)
def _fresh_planner_hint(request):
    """every GPU test starts with the planner's first-batch hint cleared
    (srtp_gpu_tune "freshmulti"): a test that plans fresh multi-SSRC
    sessions must not change which planner the next test's first batch
    takes"""
    if request.node.get_closest_marker("gpu"):
        S = sys.modules.get("re_amd.srtp")
        if S is not None:
            S.lib().srtp_gpu_tune(b"freshmulti", 0)
    yield
