"""k_long throughput vs resident waves (CLD_LONG_WAVES) on a C3/C5 batch."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = sys.argv[2] if len(sys.argv) > 2 else "50000"
for w in sys.argv[3:] or ["4", "8", "12", "16"]:
    env = dict(os.environ, CLD_LONG_WAVES=w)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--docs", n, "--steps", "3",
                          "--warmup", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=280)
    for l in out.stdout.splitlines():
        if l.startswith("{"):
            d = json.loads(l)
            print("waves/CU %s: %.0f docs/s, long kernel %.1f ms" % (w, d["value"], d["kernels"]["last_batch"]["long_ms"]),
                  flush=True)
