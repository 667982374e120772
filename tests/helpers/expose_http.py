"""Serve a Prometheus exposition callable on 127.0.0.1:<ephemeral> (tests)."""
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


def serve(expose, path: str = "/metrics"):
    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            body = expose()
            self.send_response(200 if self.path == path else 404)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, f"http://127.0.0.1:{srv.server_address[1]}{path}"
