"""Per-call cost of the zero-change drop-in (wrapper.h detect_language),
timed in C by tools/build/dl_bench: 1, 8, 64 and 256 concurrent callers each
looping over single documents, as handlers.go:132-151 calls Detect_language
once per document on concurrent goroutines.  Beside it the reference CLD2's
own per-document call (oracle/_ref/librefcld2.so, test infrastructure) on 1
and 16 threads over the same documents.  One JSON line per run.

Env: DL_RATE_CFG (c2 | c5, default both), DL_RATE_CALLERS (default 1,8,64,256),
DL_RATE_VARIANTS (";"-separated runtime environments for A/B, each one or more
","-separated K=V, e.g. "-;CLD_TINY_ZC=1;CLD_LONG_SMALL=0,CLD_MI355X_CONTEXTS=4",
"-" = as is; default "-").
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))
TABLES = os.environ.setdefault("CLD_MI355X_TABLES",
                               os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import corpus  # noqa: E402

exe = os.path.join(ROOT, "tools", "build", "dl_bench")
d = tempfile.mkdtemp()
callers_list = [int(c) for c in os.environ.get("DL_RATE_CALLERS", "1,8,64,256").split(",")]
ref_lib = os.path.join(ROOT, "oracle", "_ref", "librefcld2.so")
data_file = None
if os.path.exists(ref_lib):
    import cld2_data_file
    import cldt
    data_file = os.path.join(d, "tables.cld2_data_file00")
    with open(data_file, "wb") as f:
        f.write(cld2_data_file.build(cldt.Blob.load(TABLES)))


def run(args, timeout=300, env=None):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-3000:], file=sys.stderr)
        sys.exit(1)
    return json.loads(r.stdout.strip().splitlines()[-1])


for cfg in os.environ.get("DL_RATE_CFG", "c2,c5").split(","):
    buf, offs = corpus.GENERATORS[cfg](20000, seed=17)
    # no embedded NULs: detect_language takes C strings (wrapper.cc:8 strlen)
    assert not (buf == 0).any()
    cb, co = os.path.join(d, cfg + ".bin"), os.path.join(d, cfg + ".off")
    buf.tofile(cb)
    offs.astype(np.uint64).tofile(co)
    for var in os.environ.get("DL_RATE_VARIANTS", "-").split(";"):
        env = dict(os.environ)
        if var != "-":
            for kv in var.split(","):
                k, v = kv.split("=")
                env[k] = v
        for callers in callers_list:
            calls = max(200, 20000 // callers)
            line = run([exe, "gpu", cb, co, str(callers), str(calls)], env=env)
            line["workload"] = "%s documents, detect_language per document, %d callers" % (cfg, callers)
            line["variant"] = var
            print(json.dumps(line), flush=True)
    if data_file:
        for callers in (1, 16):
            calls = max(200, 20000 // callers) if cfg == "c2" else max(50, 2000 // callers)
            line = run([exe, "ref", ref_lib, data_file, cb, co, str(callers), str(calls)])
            line["workload"] = "%s documents, reference CLD2 per document, %d threads" % (cfg, callers)
            print(json.dumps(line), flush=True)
