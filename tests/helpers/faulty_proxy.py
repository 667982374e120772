"""A TCP proxy in front of a service that can fail on demand (KIE outage tests):

* ``pass``   -- bytes are forwarded both ways;
* ``refuse`` -- the listener is closed and every open connection is reset (connection
  refused / reset by peer: a crashed or unreachable KIE pod);
* ``503``    -- connections are accepted and every request is answered with a bare
  ``503 Service Unavailable`` (a KIE pod that is up but failing).
"""
from __future__ import annotations

import socket
import threading
import time

_R503 = b"HTTP/1.1 503 Service Unavailable\r\nContent-Length: 0\r\nConnection: close\r\n\r\n"


class FaultyProxy:
    def __init__(self, upstream_port: int, host: str = "127.0.0.1", port: int = 0):
        self.host = host
        self.upstream = (host, upstream_port)
        self.mode = "pass"
        self._lock = threading.Lock()
        self._conns = set()
        self._lsock = None
        self.port = port
        self._listen()

    def _listen(self):
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        for _ in range(100):
            try:
                s.bind((self.host, self.port))
                break
            except OSError:
                time.sleep(0.05)
        s.listen(128)
        self.port = s.getsockname()[1]
        self._lsock = s
        threading.Thread(target=self._accept, args=(s,), daemon=True).start()

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def _accept(self, ls):
        while True:
            try:
                c, _ = ls.accept()
            except OSError:
                return
            if self.mode == "503":
                threading.Thread(target=self._answer_503, args=(c,), daemon=True).start()
                continue
            try:
                u = socket.create_connection(self.upstream, timeout=5)
            except OSError:
                c.close()
                continue
            with self._lock:
                self._conns.update((c, u))
            for a, b in ((c, u), (u, c)):
                threading.Thread(target=self._pump, args=(a, b), daemon=True).start()

    def _answer_503(self, c):
        try:
            c.settimeout(2)
            c.recv(65536)
            c.sendall(_R503)
        except OSError:
            pass
        finally:
            c.close()

    def _pump(self, a, b):
        try:
            while True:
                d = a.recv(65536)
                if not d:
                    break
                b.sendall(d)
        except OSError:
            pass
        finally:
            for s in (a, b):
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                s.close()
            with self._lock:
                self._conns.discard(a)
                self._conns.discard(b)

    def _reset_all(self):
        with self._lock:
            conns = list(self._conns)
            self._conns.clear()
        for s in conns:
            try:
                s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, b"\x01\x00\x00\x00\x00\x00\x00\x00")
                s.close()
            except OSError:
                pass

    def set_mode(self, mode: str) -> None:
        assert mode in ("pass", "refuse", "503")
        prev, self.mode = self.mode, mode
        if mode in ("refuse", "503"):
            self._reset_all()
        if mode == "refuse" and self._lsock is not None:
            try:
                self._lsock.shutdown(socket.SHUT_RDWR)    # wakes the blocked accept()
            except OSError:
                pass
            self._lsock.close()
            self._lsock = None
        if prev == "refuse" and mode != "refuse":
            self._listen()

    def close(self):
        self.set_mode("refuse")
