import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RCCL_XML_DIR = "/opt/rocm/share/rccl/msccl-algorithms"
RCCL_UNIT_DIR = "/opt/rocm/share/rccl/msccl-unit-test-algorithms"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def rccl_xmls():
    import glob
    files = sorted(glob.glob(os.path.join(RCCL_XML_DIR, "*.xml")) + glob.glob(os.path.join(RCCL_UNIT_DIR, "*.xml")))
    if not files:
        pytest.skip("RCCL-shipped msccl-tools XML fixtures not present")
    return files


def xml_ngpus(path):
    import re
    with open(path) as f:
        return int(re.search(r'ngpus="(\d+)"', f.read(4096)).group(1))
