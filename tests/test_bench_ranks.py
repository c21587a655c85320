"""bench.py's multi-GPU contract on the CPU (gloo, world size 2), with only the
device work mocked (tests/bench_mock.py): `--gpus N` starts N ranks itself and
rank 0 prints one line with n_gpus N and every rank's kernel time; asking for
more GPUs than are visible, or a --gpus that disagrees with the launcher's
WORLD_SIZE, fails loudly and prints no line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--docs", "300", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-host", "--no-sub"]


def _run(gpus, visible, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CLD_BENCH_MOCK=os.path.join(ROOT, "tests", "bench_mock.py"), CLD_BENCH_MOCK_GPUS=str(visible),
               OMP_NUM_THREADS="1")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)] + ARGS,
                          capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)


def _lines(stdout):
    return [json.loads(x) for x in stdout.splitlines() if x.startswith("{")]


def test_gpus_2_runs_two_ranks_and_one_line():
    r = _run(2, 2)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "document shards, 2 rank(s)"
    pr = d["per_rank"]
    assert sorted(p["rank"] for p in pr) == [0, 1] and all(p["docs"] == 300 for p in pr)
    assert all(p["wave_ms"] > 0 for p in pr)
    # whole-job rate: both ranks' documents over the slowest rank's time
    slowest = max(p["elapsed_s"] for p in pr)
    assert abs(d["value"] - 2 * 300 * 2 / slowest) / d["value"] < 1e-6
    assert d["ms_per_step"] == slowest / 2 * 1e3


def test_more_gpus_than_visible_fails_loudly():
    r = _run(2, 1)
    assert r.returncode != 0 and not _lines(r.stdout)
    assert "GPU(s) are visible" in r.stderr


def test_gpus_must_match_launcher_world_size():
    r = _run(2, 2, {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and not _lines(r.stdout)
    assert "WORLD_SIZE" in r.stderr


def test_single_gpu_line():
    r = _run(1, 1)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _lines(r.stdout)
    assert d["n_gpus"] == 1 and d["per_rank"] is None
