"""Tracing: per-request latency records and roctx ranges.

* :class:`RequestTracer` — pass ``Client(tracer=RequestTracer())``; the
  connection records ``(xid, opcode, t_submit, t_reply, err)`` for every
  reply in a fixed-size ring; :meth:`RequestTracer.summary` gives per-opcode
  count / p50 / p99 in microseconds.  The reference only had bunyan trace
  logs per request (``lib/connection-fsm.js:361-365``, ``:396-399``).
* :func:`roctx_range` — a context manager that opens a roctx range around
  GPU codec work when ``ZKMI_ROCTX=1`` (torch's ``cuda.nvtx`` is roctx on
  ROCm), so rocprofv3 timelines show encode / frame-scan / decode phases.
"""

import contextlib
import os
import threading
import time

import numpy as np


class RequestTracer(object):

    def __init__(self, capacity=1 << 16):
        self.capacity = capacity
        self.lat_us = np.zeros(capacity, np.float64)
        self.opcode = [None] * capacity
        self.err = [None] * capacity
        self.n = 0
        self._lock = threading.Lock()

    def record(self, xid, opcode, t_submit, err):
        dt = (time.perf_counter() - t_submit) * 1e6
        with self._lock:
            k = self.n % self.capacity
            self.lat_us[k] = dt
            self.opcode[k] = opcode
            self.err[k] = err
            self.n += 1

    def summary(self):
        with self._lock:
            m = min(self.n, self.capacity)
            lat = self.lat_us[:m].copy()
            ops = list(self.opcode[:m])
        out = {}
        for op in sorted(set(o for o in ops if o is not None)):
            v = lat[[i for i, o in enumerate(ops) if o == op]]
            out[op] = {'n': int(v.size),
                       'p50_us': float(np.percentile(v, 50)),
                       'p99_us': float(np.percentile(v, 99))}
        return out


_ROCTX = os.environ.get('ZKMI_ROCTX') == '1'


@contextlib.contextmanager
def roctx_range(name):
    if not _ROCTX:
        yield
        return
    import torch
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
