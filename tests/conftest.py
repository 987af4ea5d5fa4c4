import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the tests drive the engine's A/B and diagnostic switches (KB_FUSE, KB_PAIR_WAIT_TICKS, ...):
# the library reads them only after this opt-in (include/kbengine.h, kb_set_diagnostics)
os.environ["KB_DIAGNOSTICS"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running parity case")


@pytest.fixture(scope="session", autouse=True)
def _build_oracle():
    from oracle import oracle
    if not os.path.exists(oracle._LIB_PATH):
        oracle.build()
    yield
