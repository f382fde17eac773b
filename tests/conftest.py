import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
PKG = ROOT / "movie-recommender-system-with-gnns_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size parity (minutes on the CPU oracle side)")


@pytest.fixture
def tune():
    """tune(field=value, ...): lgcn_amd.tuning.set_tuning for one test, the previous record restored
    after it (the path reads no environment variables)."""
    import dataclasses

    from lgcn_amd import tuning

    saved = tuning.get()
    yield tuning.set_tuning
    tuning.set_tuning(**dataclasses.asdict(saved))


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("this test is marked gpu and needs a ROCm device (run the CPU suite with -m 'not gpu')")
    return torch.device("cuda:0")
