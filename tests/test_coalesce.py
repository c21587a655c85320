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


@pytest.fixture(scope="module")
def sim_sanitized():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "build/coalesce_sim_tsan",
                    "build/coalesce_sim_asan"], check=True)
    return {k: os.path.join(ROOT, "tools", "build", "coalesce_sim_" + k) for k in ("tsan", "asan")}


@pytest.mark.parametrize("san,callers,spin,wake", [("tsan", 64, 50, "tree"), ("tsan", 32, 0, "direct"),
                                                   ("asan", 128, 0, "direct"), ("asan", 64, 50, "tree")])
def test_mixed_requests_under_sanitizers(sim_sanitized, san, callers, spin, wake):
    """Tiny and non-tiny requests with two flag values, each request a heap
    object freed the moment submit() returns: a poster still touching it (the
    round-5 post()/park() race) is a report from ThreadSanitizer or
    AddressSanitizer.  Non-tiny requests must not starve behind tiny groups."""
    r = subprocess.run([sim_sanitized[san], str(callers), "40", "30", "sleep", "1", "2", str(spin), wake, "mixed"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr, r.stdout + r.stderr[-4000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["wrong"] == 0 and d["calls"] == callers * 40 and d["non_tiny_calls"] == callers // 4 * 40
    # a non-tiny request waits for at most a few groups, not for the tiny stream to dry up
    assert d["non_tiny_latency_us_p99"] < 4 * d["latency_us_p99"] + 20000


# detect_language's per-call queue (language-detector_amd/csrc/cld_dlqueue.h)
# with a mock dispatch (tools/dlqueue_sim.cpp): lock-free stack, futex waits,
# binary-tree wake-ups, dispatcher stop requests.

@pytest.fixture(scope="module")
def dlsim():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "build/dlqueue_sim", "build/dlqueue_sim_asan",
                    "build/dlqueue_sim_tsan"], check=True)
    return {k: os.path.join(ROOT, "tools", "build", "dlqueue_sim" + k) for k in ("", "_asan", "_tsan")}


@pytest.mark.parametrize("callers,dispatchers,cspin,dspin", [(1, 2, 30, 100), (8, 2, 30, 100), (64, 2, 30, 0),
                                                             (256, 2, 0, 100), (256, 4, 30, 0)])
def test_dl_queue_every_caller_gets_its_own_result(dlsim, callers, dispatchers, cspin, dspin):
    calls = max(20, 8000 // callers)
    r = subprocess.run([dlsim[""], str(callers), str(calls), str(dispatchers), "30", str(cspin), str(dspin)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["wrong"] == 0 and d["calls"] == callers * calls
    if callers >= 64:
        assert d["docs_per_batch"] > 2          # calls that arrive during a launch share the next one


@pytest.mark.parametrize("san,callers,dispatchers,cspin,dspin", [("_tsan", 64, 2, 30, 100), ("_tsan", 16, 1, 0, 0),
                                                                 ("_asan", 128, 3, 0, 0), ("_asan", 32, 2, 30, 50)])
def test_dl_queue_under_sanitizers(dlsim, san, callers, dispatchers, cspin, dspin):
    """Each request is a heap object freed the moment wait() returns: a
    dispatcher or a wake-up parent still touching it is a report."""
    r = subprocess.run([dlsim[san], str(callers), "40", str(dispatchers), "20", str(cspin), str(dspin)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr, r.stdout + r.stderr[-4000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["wrong"] == 0 and d["calls"] == callers * 40
