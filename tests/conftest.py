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


def pytest_collection_modifyitems(session, config, items):
    # the full-size reference sweep (test_gpu_zfullsize.py, last in the GPU
    # suite) needs minutes of corpus generation: start it in the background
    # as soon as the session knows it will run
    if any(it.get_closest_marker("gpu") and "zfullsize" in it.nodeid for it in items):
        import fullsize
        fullsize.prefetch()


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


@pytest.fixture(scope="module", params=["q1", "q0"])
def ref_tables(request, gpu, tmp_path_factory):
    """(label, reference CLD2 instance) with the GPU and the reference on the same
    tables: the synthetic Q1 (the suite's default), then the product's shipped Q0,
    loaded on both sides through the cld2 data-file loaders (cld_load_data_from_file
    / the reference's loadDataFromFile); the GPU gets Q1 back afterwards."""
    import refcld
    refcld.verify_build()
    if request.param == "q1":
        yield "q1", refcld.instance(os.environ["CLD_MI355X_TABLES"])
        return
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import cld2_data_file
    import cldt
    q0 = os.path.join(ROOT, "language-detector_amd", "data", "cld2_q0.cldt")
    p = tmp_path_factory.mktemp("q0") / "q0.cld2_data_file00"
    p.write_bytes(cld2_data_file.build(cldt.Blob.load(q0)))
    gpu.load_data_from_file(str(p))
    try:
        yield "q0", refcld.instance(q0)
    finally:
        gpu.unload_data()
