"""Throughput of the batch HTTP route (language-detector_amd/service.py) on
C5-shaped requests: texts drawn from corpus.c5 (lognormal lengths, mixed
scripts), packed into POST / bodies of at most 1 MB (the reference's body
limit, main.go:32), each answered by ONE cld_detect_batch call with
StripExtras + C-string preparation on the GPU.

Two figures, both docs/s: in-process (LanguageDetectorService.handle: JSON
parse + GPU batch + JSON response) and over HTTP on 127.0.0.1 (the stdlib
threading server, CLIENTS concurrent keep-alive clients).  Prints one JSON line.

    python tools/service_rate.py [--docs N] [--seconds S] [--clients C]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))


def bodies(n, limit=1048576):
    import corpus
    buf, offs = corpus.c5(n, seed=0xC1D2_0505)
    out, cur, size, docs = [], [], 20, []
    for i in range(n):
        t = bytes(buf[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
        item = json.dumps({"text": t}, ensure_ascii=False)
        b = len(item.encode()) + 1
        if cur and size + b > limit - 64:
            out.append(('{"request":[' + ",".join(cur) + "]}").encode())
            docs.append(len(cur))
            cur, size = [], 20
        cur.append(item)
        size += b
    if cur:
        out.append(('{"request":[' + ",".join(cur) + "]}").encode())
        docs.append(len(cur))
    return out, docs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=200_000)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--clients", type=int, default=8)
    a = ap.parse_args()
    import cld_amd
    import service
    cld_amd.init_device(0)
    known = json.load(open(os.path.join(ROOT, "tests", "golden", "main_test.json")))["known_languages"]
    svc = service.LanguageDetectorService(known)
    reqs, ndocs = bodies(a.docs)
    svc.handle("POST", "/", "application/json", reqs[0])        # warm
    res = {"requests": len(reqs), "docs_per_request_mean": sum(ndocs) / len(ndocs),
           "body_bytes_mean": sum(map(len, reqs)) / len(reqs)}
    # in process
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        for r, k in zip(reqs, ndocs):
            st, out = svc.handle("POST", "/", "application/json", r)
            assert st in (200, 203), st
            done += k
    dt = time.perf_counter() - t0
    res["in_process_docs_per_s"] = done / dt
    # over HTTP, keep-alive clients
    import http.client
    srv = service.make_server(svc, 0, "127.0.0.1")
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    counts = [0] * a.clients
    stop = time.perf_counter() + a.seconds

    def client(c):
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        j = c
        while time.perf_counter() < stop:
            conn.request("POST", "/", body=reqs[j % len(reqs)], headers={"Content-Type": "application/json"})
            r = conn.getresponse()
            r.read()
            assert r.status in (200, 203), r.status
            counts[c] += ndocs[j % len(reqs)]
            j += a.clients
    th = [threading.Thread(target=client, args=(c,)) for c in range(a.clients)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    srv.shutdown()
    res["http_docs_per_s"] = sum(counts) / dt
    res["http_clients"] = a.clients
    res["unit"] = "docs/s"
    res["workload"] = "C5-shaped texts (corpus.c5), <= 1 MB JSON bodies, POST / with StripExtras + C-string cut"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
