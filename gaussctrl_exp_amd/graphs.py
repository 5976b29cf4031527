"""One training (or render) step of the fused path captured as a HIP graph and replayed.

The fused step issues ~25 kernels through ~10 C-ABI calls plus torch's autograd between them;
on small frames (c3: 512x512, ~0.3 ms of kernels) the host's Python/ctypes work per step is
as long as the GPU's, so the GPU idles between launches.  Since the speculative binning
(rasterize.SpeculativeBinning) took the host read of I out of the step, the whole step -- the
fused preprocess, the binning, the blend with the L1 loss, the raster backward and the fused
preprocess backward -- is a fixed launch sequence on one stream for a given frame shape and
capacity, so it is captured once (torch.cuda.graph: every launch our C-ABI issues goes to the
capturing stream) and replayed as one graph launch per step.

What stays on the host per replay: the check of the binning's pinned count words
(SpeculativeBinning.check_replay), written by the emission kernel early in the step while the
GPU carries on.  A replay whose intersection count exceeded the captured capacity rendered from
an empty table; replay() then returns False, the owner re-runs the step eagerly (which re-bins)
and the graph is captured again at the new capacity on the next call.  (A captured binning
assumes no constant depth digit, so a changing depth range cannot invalidate a replay.)
Replays read the step's inputs from the tensors they were captured with (parameters, camera,
ground truth, background): update those in place.

Measured on MI355X / ROCm 7: replaying is slower than issuing the same launches
from the stream (headline 0.761 vs 0.748 ms per step, c3 0.403 vs 0.392), so bench.py issues
eagerly unless --graph on.

A training step with the in-backward Adam is replayable too when its schedule lives on the
device (TrainStep.step(device_schedule=True): the learning rates and bias corrections from a
table indexed by a device step counter, and the Adam kernel itself skips the update when the
binning's device count word says the replay overflowed), with after_capture / after_replay
keeping the host's step count in step.

Single GPU only (the N > 1 step's collectives stay eager).  Reference step:
gaussctrl/gc_pipeline.py:469-480 (loss, backward per view) around gc_model.py:158-222.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch

from . import fused
from .rasterize import GraphCaptureUnsupported


class StepGraph:
    """fn() -- one step on the current device -- as a replayable HIP graph.

    params: tensors whose .grad the step assigns (autograd leaves); after each replay their
    .grad are the graph's gradient tensors again (an eager fallback replaces them)."""

    def __init__(self, fn: Callable[[], object], device, params: Sequence[torch.Tensor] = (),
                 warmup: int = 1, after_capture: Optional[Callable[[], None]] = None,
                 after_replay: Optional[Callable[[], None]] = None):
        self.fn = fn
        # host bookkeeping of a step whose effects live on the device (a training step's step
        # count: TrainStep.advance_step_count): undone after the capture (which ran nothing),
        # redone after each valid replay
        self.after_capture = after_capture
        self.after_replay = after_replay
        self.dev = torch.device(device)
        self.params = list(params)
        self.warmup = warmup
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.specs: List = []
        self.grads: List[Optional[torch.Tensor]] = []
        self.result = None
        self.replays = 0
        self.fallbacks = 0
        self.captures = 0
        self.unsupported: Optional[str] = None
        self.warm_result = None
        self.warm_grads: List[Optional[torch.Tensor]] = []

    # ------------------------------------------------------------------ capture
    def capture(self) -> bool:
        """Warm up eagerly (capacity, key range, autograd and allocator state: `warmup` real
        steps, the last one's result kept in .warm_result), then capture (which runs nothing).
        False (and the reason in .unsupported) when the step needs a host read of I."""
        self.close()
        cur = torch.cuda.current_stream(self.dev)
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(max(self.warmup, 1)):
                self.warm_result = self.fn()
        cur.wait_stream(side)
        # the warm-up step's gradients (the capture below assigns the graph's own, unexecuted)
        self.warm_grads = [p.grad for p in self.params]
        mode = fused.LAST_BINNING["mode"]
        if mode != "speculative":
            # "sync": the frame shape's first binning (no capacity known yet) -- the next call
            # tries again; "host": a scheme that reads I on the host -- never capturable
            if mode == "host":
                self.unsupported = "binning mode 'host'"
            return False
        for p in self.params:
            p.grad = None
        g = torch.cuda.CUDAGraph()
        specs: list = []
        fused._CAPTURE_SPECS = specs
        try:
            with torch.cuda.graph(g):
                result = self.fn()
        except GraphCaptureUnsupported as e:
            for s in specs:
                s.release()
            self.unsupported = str(e)
            return False
        finally:
            fused._CAPTURE_SPECS = None
        if self.after_capture is not None:
            self.after_capture()
        if not specs:
            self.unsupported = "the step launched no speculative binning"
            return False
        self.graph, self.specs, self.result = g, specs, result
        self.grads = [p.grad for p in self.params]
        self.captures += 1
        self.unsupported = None
        return True

    def close(self):
        for s in self.specs:
            s.release()
        self.specs, self.graph, self.result, self.grads = [], None, None, []

    # ------------------------------------------------------------------ replay
    def replay(self) -> bool:
        """One step.  True: the replay's outputs (.result, the params' .grad) are valid.
        False: they are not (capacity overflow / depth-range violation); run the step eagerly
        -- step() does -- and the next call captures again."""
        if self.graph is None:
            raise RuntimeError("StepGraph.replay: nothing captured")
        self.graph.replay()
        stream = torch.cuda.current_stream(self.dev)
        ok = True
        for s in self.specs:
            ok = s.check_replay(stream) and ok
        self.replays += 1
        if ok:
            for p, g in zip(self.params, self.grads):
                p.grad = g
            if self.after_replay is not None:
                self.after_replay()
        return ok

    def step(self):
        """One step: a replay, or -- when nothing is captured yet -- the warm-up (its last eager
        step is this call's step) and the capture; an invalid replay is redone eagerly and the
        graph dropped so the next step captures again.  Returns the step's result.  With
        warmup = 1 every call is exactly one step (a training loop's step count holds)."""
        if self.graph is None and self.unsupported is None:
            self.capture()
            if self.warmup <= 1 or self.graph is None:
                for p, g in zip(self.params, self.warm_grads):
                    p.grad = g
                return self.warm_result
            # (more warm-up steps than one: the calls before the capture were extra steps)
        if self.graph is None:
            return self.fn()
        if self.replay():
            return self.result
        self.fallbacks += 1
        self.close()
        for p in self.params:
            p.grad = None
        return self.fn()

    def stats(self) -> dict:
        return {"replays": self.replays, "fallbacks": self.fallbacks,
                "captures": self.captures, "unsupported": self.unsupported}
