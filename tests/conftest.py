import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "kmer-ml_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def edge_cases():
    import json
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def synthetic_cases():
    import json
    with open(os.path.join(GOLDEN, "synthetic.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def oracle_lib():
    """Build (if needed) and load the C restatement."""
    import subprocess
    lib = os.path.join(REPO, "oracle", "build", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    from oracle import corac
    return corac
