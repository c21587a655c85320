"""The request coalescer (language-detector_amd/csrc/cld_coalesce.h) on the
host, with a mock dispatch (tools/coalesce_sim.cpp): every caller gets exactly
its own results, at 1 to 256 concurrent callers, with and without the spin
before parking, with tree and direct wake-ups.  No GPU."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, "tools", "build", "coalesce_sim")


@pytest.fixture(scope="module")
def sim():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "build/coalesce_sim"], check=True)
    return SIM


@pytest.mark.parametrize("callers,spin,wake", [(1, 0, "tree"), (8, 0, "tree"), (64, 50, "tree"), (256, 0, "tree"),
                                               (256, 50, "direct"), (128, 50, "tree")])
def test_every_caller_gets_its_own_results(sim, callers, spin, wake):
    calls = max(20, 4000 // callers)
    r = subprocess.run([sim, str(callers), str(calls), "30", "sleep", "1", "2", str(spin), wake],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["wrong"] == 0 and d["calls"] == callers * calls
    if callers >= 64:
        assert d["docs_per_group"] > 2          # requests did coalesce
