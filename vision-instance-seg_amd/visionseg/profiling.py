"""Per-kernel HIP-event timing of the hand-written ops (used by bench.py's roofline).

`timed(name, tensor, bytes_=, flops=)` brackets one C-ABI launch with two
`torch.cuda.Event`s recorded on the stream the kernel is launched on (the inputs'
current stream — the same stream the ops pass to the C ABI) and records the launch's
ALGORITHMIC work (compulsory HBM bytes and/or useful flops, computed from the shapes).
Disabled (one global check) unless a `KernelTimer` is active.

Eager steps are host-bound (the host enqueues slower than the GPU drains), so a start
event recorded on an idle stream would also time the host's op preparation.  With
`spin` (default) a short device spin (`torch.cuda._sleep`) is enqueued before the start
event: the GPU is still busy with it while the host enqueues the event and the op, so the
pair brackets only the op's kernels.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch

_active = None


_SPIN_CYCLES = 200_000   # ~0.1 ms of device clock: longer than one op's host-side enqueue


class KernelTimer:
    def __init__(self, spin: bool = True):
        self.events = defaultdict(list)
        self.spin = spin

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
        """{name: dict(launches, total_ms, mean_ms, bytes, flops)} — call after a sync.
        bytes/flops are per-launch averages of the algorithmic work."""
        out = {}
        for name, evs in self.events.items():
            ts = [a.elapsed_time(b) for a, b, _, _ in evs]
            n = len(ts)
            out[name] = dict(launches=n, total_ms=sum(ts), mean_ms=sum(ts) / max(1, n),
                             bytes=sum(x[2] for x in evs) / max(1, n), flops=sum(x[3] for x in evs) / max(1, n))
        return out


def enabled() -> bool:
    return _active is not None


@contextlib.contextmanager
def timed(name: str, like: torch.Tensor, bytes_: float = 0.0, flops: float = 0.0):
    t = _active
    if t is None:
        yield
        return
    s = torch.cuda.current_stream(like.device)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    if t.spin:
        with torch.cuda.stream(s):
            torch.cuda._sleep(_SPIN_CYCLES)
    a.record(s)
    try:
        yield
    finally:
        b.record(s)
        t.events[name].append((a, b, float(bytes_), float(flops)))
