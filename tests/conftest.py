import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLD


@pytest.fixture(scope="session")
def sai_manifest():
    with open(os.path.join(GOLD, "sai_manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_index():
    import oracle
    return oracle.Bwt(os.path.join(GOLD, "g1m.bwt")), oracle.Bwt(os.path.join(GOLD, "g1m.rbwt"))


@pytest.fixture(scope="session")
def gpu_engine():
    from ibwa_amd.engine import Engine
    eng = Engine(0)
    eng.load_index_files(os.path.join(GOLD, "g1m"))
    yield eng
    eng.close()
