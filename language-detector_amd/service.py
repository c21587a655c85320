"""The service's request handling over the batch entry point.

Mirrors the reference's HTTP surface for the detection path -- routes, JSON
shapes, status codes and error texts -- with one change of mechanism: every
text of a request is prepared and scored in ONE cld_detect_batch call on the
GPU (StripExtras + C-string cut + DetectLanguage), instead of one cgo call per
item.
  routes            main.go:185-191 getRouter: GET / usage, POST / detect, else 404
  usage / 404       main.go:29-51 USAGE_STRING, main.go:165-181 GenerateResponses
  request parsing   handlers.go:31-67 GetRequests (Content-Type, 1 MB body limit, JSON)
  POST /            handlers.go:105-183 LanguageDetectorHandler
  per item          handlers.go:150-151 StripExtras + Detect_language, names from
                    data/cld_codes.json (main.go:114-124: the deployer's file)
Prometheus counters and bunyan logging (main.go:134-240) are the service's
control plane and stay out of scope.

`LanguageDetectorService.handle(method, path, content_type, body)` returns
(status, body bytes); `serve()` puts it behind the standard library's
threading HTTP server for manual use.
"""
import json

import cld_amd

BODY_LIMIT_BYTES = 1048576     # main.go:32
DRAIN_LIMIT = 64 << 20         # an oversized body's remainder is read and discarded up to this
CONTENT_TYPE_OUT = "application/json; charset=utf-8"

USAGE = {"result": {"id": "language-detector", "name": "language-detector",
                    "description": "Determine language code from text",
                    "in": {"text": {"type": "string"}},
                    "out": {"iso6391code": {"type": "string"}, "name": {"type": "string"}}}}


def _dump(obj):
    """rapidjson's compact writer: no whitespace, UTF-8 kept as is."""
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False).encode("utf-8")


def _reject_constant(name):
    """rapidjson (kParseDefaultFlags) rejects NaN / Infinity / -Infinity; so must we."""
    raise ValueError("non-standard JSON constant %s" % name)


def _first_key_object(pairs):
    d = {}
    for k, v in pairs:              # rapidjson GetMember finds the first member of a name
        d.setdefault(k, v)
    return d


def gpu_detect_codes(texts):
    """Raw request texts -> ISO codes, as handlers.go:150-151 + main.go:77-81 compute them,
    in one batch: prepare (StripExtras, C-string cut) and detect on the GPU."""
    if not texts:
        return []
    res = cld_amd.detect_batch(docs=texts, flags=cld_amd.FLAG_STRIP_EXTRAS | cld_amd.FLAG_CSTRING)
    return [cld_amd.result_code(r) for r in res]


class LanguageDetectorService:
    def __init__(self, known_languages, detect_codes=gpu_detect_codes, body_limit=BODY_LIMIT_BYTES):
        self.known = dict(known_languages)
        self.detect_codes = detect_codes
        self.body_limit = body_limit
        self.usage = _dump(USAGE)
        self.not_found = _dump({"error": "Not found"})

    @classmethod
    def from_file(cls, lang_file, **kw):
        """main.go:114-124: known languages from a JSON object code -> name."""
        with open(lang_file, "rb") as f:
            return cls(json.loads(f.read().decode("utf-8")), **kw)

    @staticmethod
    def _error(message, status):
        return status, _dump({"error": message})            # handlers.go:14-28

    def handle(self, method, path, content_type, body):
        if path == "/" and method == "GET":
            return 200, self.usage
        if path == "/" and method == "POST":
            return self._detect(content_type, body)
        return 404, self.not_found

    def _detect(self, content_type, body):
        # GetRequests (handlers.go:31-67)
        if content_type != "application/json":
            return self._error("Content-Type must be set to application/json", 400)
        body = bytes(body[:self.body_limit])
        try:
            doc = json.loads(body.decode("utf-8", "surrogateescape"), object_pairs_hook=_first_key_object,
                             parse_constant=_reject_constant)
        except ValueError:
            return self._error("Unable to parse request - invalid JSON detected", 400)
        if doc is None:                                       # handlers.go:112-114: nothing written
            return 200, b""
        if not isinstance(doc, dict) or "request" not in doc:
            return self._error("Unable to parse request - invalid JSON detected", 400)
        requests = doc["request"] if isinstance(doc["request"], list) else []
        # gather every text of the request, one batch
        items, texts = [], []
        for req in requests:
            if not isinstance(req, dict) or "text" not in req:
                items.append(None)
                continue
            t = req["text"]
            if not isinstance(t, str):
                t = ""                                        # GetString on a non-string: ""
            try:
                texts.append(t.encode("utf-8", "surrogateescape"))
            except UnicodeEncodeError:                        # a lone \\uD8xx escape: rapidjson rejects it
                return self._error("Unable to parse request - invalid JSON detected", 400)
            items.append(len(texts) - 1)
        codes = self.detect_codes(texts)
        status = 200
        out = []
        for it in items:                                      # handlers.go:133-176, in request order
            if it is None:
                out.append({"error": "Missing text key"})
                status = 400
                continue
            code = codes[it]
            name = self.known.get(code)
            if name is None:
                name = "Unknown"
                status = 203
            out.append({"iso6391code": code, "name": name})
        return status, _dump({"response": out})


def make_server(service, port=3000, host=""):
    """HTTP server around `service.handle` (stdlib, one thread per connection)."""
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    class H(BaseHTTPRequestHandler):
        def _reply(self, method):
            n = int(self.headers.get("Content-Length") or 0)
            # io.LimitReader (handlers.go:40): never read past the limit
            body = self.rfile.read(min(n, service.body_limit)) if n > 0 else b""
            # the rest of an oversized body: discard it (up to DRAIN_LIMIT) so
            # the reply is not lost to a reset when the socket closes with
            # unread data, as net/http does; beyond that, close after replying
            left = n - len(body)
            close = False
            while left > 0:
                if n - service.body_limit > DRAIN_LIMIT:
                    close = True
                    break
                got = self.rfile.read(min(left, 1 << 16))
                if not got:
                    break
                left -= len(got)
            status, out = service.handle(method, self.path, self.headers.get("Content-Type", ""), body)
            self.send_response(status)
            if out or status != 200:
                self.send_header("Content-Type", CONTENT_TYPE_OUT)
            self.send_header("Content-Length", str(len(out)))
            if close:
                self.send_header("Connection", "close")
                self.close_connection = True
            self.end_headers()
            self.wfile.write(out)
            if close:
                import socket
                self.wfile.flush()
                try:
                    self.connection.shutdown(socket.SHUT_WR)
                except OSError:
                    pass

        def do_GET(self):
            self._reply("GET")

        def do_POST(self):
            self._reply("POST")

        def log_message(self, *a):
            pass

    return ThreadingHTTPServer((host, port), H)


def serve(service, port=3000):
    """Blocking HTTP server around `service.handle`."""
    make_server(service, port).serve_forever()
