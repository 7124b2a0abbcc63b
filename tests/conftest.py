import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "kubernetes-native-distributed-ai-job-scheduler_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# The library's A/B and test knobs (KP_FUSED, KP_FZ_TIE_BITS, ...) are read
# only under KP_DEBUG_KNOBS=1; the tests that set one exercise alternative
# code paths on purpose (tests/test_gpu_parity.py), so the suite opts in.
os.environ["KP_DEBUG_KNOBS"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle_bind
    oracle_bind.build()
    return oracle_bind


@pytest.fixture(scope="session")
def placer():
    from kplace.engine import Placer
    p = Placer(device=0)
    yield p
    p.close()
