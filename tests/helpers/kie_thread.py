"""The KIE REST server (process/kie_server.py) on its own event-loop thread: a separate
'pod' for hand-off / outage tests."""
import asyncio
import threading

from ccfd_demo_summit_amd.process.kie_server import KieServer


class KieThread:
    """The aiohttp KIE server on its own event-loop thread (a separate 'pod')."""

    def __init__(self, engine):
        from aiohttp import web
        self.srv = KieServer(engine, tick_s=0.05)
        self.loop = asyncio.new_event_loop()
        self.runner = web.AppRunner(self.srv.app)
        ready = threading.Event()

        def run():
            asyncio.set_event_loop(self.loop)
            self.loop.run_until_complete(self.runner.setup())
            site = web.TCPSite(self.runner, "127.0.0.1", 0)
            self.loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            ready.set()
            self.loop.run_forever()
        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()
        assert ready.wait(10)

    def close(self):
        fut = asyncio.run_coroutine_threadsafe(self.runner.cleanup(), self.loop)
        fut.result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
