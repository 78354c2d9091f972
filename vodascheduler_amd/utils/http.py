"""Minimal threaded HTTP server + router (stdlib only) used by the three REST services."""
from __future__ import annotations

import json
import logging
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable

log = logging.getLogger("vodascheduler_amd.http")

# handler(body: bytes, query: str) -> (status, content_type, payload bytes)
Handler = Callable[[bytes, str], tuple[int, str, bytes]]


def text(status: int, s: str) -> tuple[int, str, bytes]:
    return status, "text/plain; charset=utf-8", s.encode()


def as_json(status: int, obj) -> tuple[int, str, bytes]:
    return status, "application/json", json.dumps(obj).encode()


class Router:
    def __init__(self):
        self.routes: dict[tuple[str, str], Handler] = {}

    def add(self, method: str, path: str, fn: Handler) -> None:
        self.routes[(method.upper(), path)] = fn


class HttpServer:
    def __init__(self, router: Router, host: str = "0.0.0.0", port: int = 0, name: str = "voda"):
        routes = router.routes

        class _H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def _dispatch(self, method: str):
                path, _, query = self.path.partition("?")
                fn = routes.get((method, path))
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                if fn is None:
                    status, ctype, payload = text(404, f"404 page not found: {method} {path}\n")
                else:
                    try:
                        status, ctype, payload = fn(body, query)
                    except Exception as e:  # never kill the server thread
                        log.exception("handler error")
                        status, ctype, payload = text(500, f"internal error: {e}\n")
                self.send_response(status)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(payload)))
                self.end_headers()
                self.wfile.write(payload)

            def do_GET(self):
                self._dispatch("GET")

            def do_POST(self):
                self._dispatch("POST")

            def do_PUT(self):
                self._dispatch("PUT")

            def do_DELETE(self):
                self._dispatch("DELETE")

            def log_message(self, fmt, *args):
                log.debug("%s " + fmt, name, *args)

        self.httpd = ThreadingHTTPServer((host, port), _H)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self._thread: threading.Thread | None = None

    def start(self) -> "HttpServer":
        self._thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self._thread.start()
        return self

    def serve_forever(self) -> None:
        self.httpd.serve_forever()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def http_request(method: str, url: str, body: bytes | None = None, timeout: float = 30.0,
                 content_type: str = "application/json") -> tuple[int, bytes]:
    import urllib.error
    import urllib.request

    req = urllib.request.Request(url, data=body, method=method, headers={"Content-Type": content_type})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, r.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()
