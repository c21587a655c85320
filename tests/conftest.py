import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tools", ""):
    sys.path.insert(0, os.path.join(ROOT, p))

# The library's default tables are Q0 (empty quadgram table).  The parity
# suite opts into the synthetic Q1 table explicitly, so the quadgram path is
# exercised; the oracle reads the same file (oracle.DEFAULT_TABLES).
os.environ.setdefault("CLD_MI355X_TABLES",
                      os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP path)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu():
    import cld_amd
    cld_amd.init()
    return cld_amd


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "cld2_unittest.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def verbose_golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "cld2_verbose.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "main_test.json"), encoding="utf-8") as f:
        return json.load(f)["kats"]


@pytest.fixture(scope="session")
def blob():
    import cldt
    return cldt.Blob.load(os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
