"""Per-entry-point HIP-event timing of the C-ABI calls (used by bench.py).

When enabled, every `_lib.call` is bracketed by two events recorded on the stream the
kernels are launched on (torch's current stream, which is what the wrappers pass to the
C ABI), so per-call device durations are measured live without a profiler.
"""
from __future__ import annotations

import collections
import contextlib

import torch

from . import _lib

_orig_call = _lib.call
_orig_call_status = _lib.call_status


class CallTimer:
    def __init__(self):
        self.events = collections.defaultdict(list)

    def _call(self, name, *args, _fn=None):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        # a call issued on another stream than the current one (the fused forward's colour
        # part, concurrent with the binning): bracketed on that stream, and keyed apart
        st = args[-1] if args and isinstance(args[-1], int) else None
        side = st is not None and st != torch.cuda.current_stream().cuda_stream
        ext = torch.cuda.ExternalStream(st) if side else None
        s.record(ext)
        rc = (_fn or _orig_call)(name, *args)
        e.record(ext)
        # the list-split variants are the same entry (gsplat_rasterize_forward/_backward)
        key = name[:-len("_chunked")] if name.endswith("_chunked") else name
        if name == "gsplat_fused_preprocess_forward_part":
            key = f"{name}[{args[0]}]"
        if side:
            key += " (side stream)"
        self.events[key].append((s, e))
        return rc

    def summary(self):
        """{name: (calls, mean_ms, total_ms)} -- synchronises the device."""
        torch.cuda.synchronize()
        out = {}
        for name, evs in self.events.items():
            ms = [s.elapsed_time(e) for s, e in evs]
            out[name] = (len(ms), sum(ms) / len(ms), sum(ms))
        return out


@contextlib.contextmanager
def timed_calls():
    t = CallTimer()
    _lib.call = t._call
    _lib.call_status = lambda name, *a: t._call(name, *a, _fn=_orig_call_status)
    try:
        yield t
    finally:
        _lib.call = _orig_call
        _lib.call_status = _orig_call_status
