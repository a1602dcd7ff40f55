"""Wall-clock ``Timer`` with the interface of ``custma.Timer``
(reference: custma/utils.py:13-87): ``Timer(print_tmpl=None, start=True)``,
context manager printing the elapsed seconds, ``start()``, ``since_start()``,
``since_last_check()``, ``is_running``, ``TimerError``.

Like the reference it measures host wall time.  Unlike the reference it can
synchronise the device (``sync=True``) so the number is kernel time rather
than launch latency; the default is off for drop-in compatibility.  For real
measurements use bench.py (HIP events).
"""
from __future__ import annotations

import re
import time


class TimerError(Exception):
    def __init__(self, message):
        self.message = message
        super().__init__(message)


class Timer:
    def __init__(self, print_tmpl=None, start=True, sync=False):
        self._running = False
        self.sync = sync
        if print_tmpl is not None and not re.search(r"\{:.*\d+f\}", print_tmpl):
            print_tmpl = print_tmpl + " {:.3f}"
        self.print_tmpl = print_tmpl or "{:.3f}"
        if start:
            self.start()

    def _now(self):
        if self.sync:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
        return time.time()

    @property
    def is_running(self):
        return self._running

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, exc_type, exc, tb):
        print(self.print_tmpl.format(self.since_last_check()))
        self._running = False

    def start(self):
        if not self._running:
            self._t_start = self._now()
            self._running = True
        self._t_last = self._now()

    def since_start(self):
        if not self._running:
            raise TimerError("timer is not running")
        self._t_last = self._now()
        return self._t_last - self._t_start

    def since_last_check(self):
        if not self._running:
            raise TimerError("timer is not running")
        now = self._now()
        dur = now - self._t_last
        self._t_last = now
        return dur
