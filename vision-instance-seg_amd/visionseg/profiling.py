"""Per-kernel HIP-event timing of the hand-written ops (used by bench.py's roofline).

`timed(name, tensor)` brackets one C-ABI launch with two `torch.cuda.Event`s recorded
on the stream the kernel is launched on (the inputs' current stream — the same stream
the ops pass to the C ABI).  Disabled (zero overhead beyond a flag check) unless a
`KernelTimer` is active.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch

_active = None


class KernelTimer:
    def __init__(self):
        self.events = defaultdict(list)

    def __enter__(self):
        global _active
        self._prev = _active
        _active = self
        return self

    def __exit__(self, *exc):
        global _active
        _active = self._prev
        return False

    def summary(self):
        """{name: (launches, total_ms, mean_ms)} — call after synchronising."""
        out = {}
        for name, evs in self.events.items():
            ts = [a.elapsed_time(b) for a, b in evs]
            out[name] = (len(ts), sum(ts), sum(ts) / max(1, len(ts)))
        return out


@contextlib.contextmanager
def timed(name: str, like: torch.Tensor):
    t = _active
    if t is None:
        yield
        return
    s = torch.cuda.current_stream(like.device)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    try:
        yield
    finally:
        b.record(s)
        t.events[name].append((a, b))
