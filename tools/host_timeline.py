"""Where the host spends a bench step: perf_counter stamps around every C-ABI call
(_lib.call / call_status), the binning's wait for the intersection count (_wait_count) and
the step's phases (zero_grad, forward, backward), averaged over STEPS steady-state steps and
printed as offsets from the step's start.  CFG selects the bench config (default c3)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
from gaussctrl_exp_amd import _lib, rasterize
from gaussctrl_exp_amd.train import TrainStep

cfg = os.environ.get("CFG", "c3")
steps = int(os.environ.get("STEPS", "200"))
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
scene, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
H, W = cam.height, cam.width
gt = torch.rand(H, W, 3, device=dev)
bg = torch.zeros(3, device=dev)
tr = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")

events = []
clock = time.perf_counter


def wrap(fn, label):
    def w(name, *a):
        t0 = clock()
        r = fn(name, *a)
        events.append((f"{label} {name}", t0, clock()))
        return r
    return w


def wrap_plain(fn, label):
    def w(*a, **k):
        t0 = clock()
        r = fn(*a, **k)
        events.append((label, t0, clock()))
        return r
    return w


_lib.call = wrap(_lib.call, "call")
_lib.call_status = wrap(_lib.call_status, "call_status")
rasterize._wait_count = wrap_plain(rasterize._wait_count, "wait I")
# small host calls, summed per step (count, time)
small = collections.defaultdict(lambda: [0, 0.0])


def wrap_small(fn, label):
    def w(*a, **k):
        t0 = clock()
        r = fn(*a, **k)
        e = small[label]
        e[0] += 1
        e[1] += clock() - t0
        return r
    return w


torch.empty = wrap_small(torch.empty, "torch.empty")
_lib.query = wrap_small(_lib.query, "_lib.query")
_lib.check_device = wrap_small(_lib.check_device, "_lib.check_device")
_lib.stream = wrap_small(_lib.stream, "_lib.stream")


FWD_ONLY = cfg in bench.FORWARD_ONLY or os.environ.get("FWD_ONLY") == "1"


def step():
    t0 = clock()
    if FWD_ONLY:  # bench.py's forward-only step (c2): the fused render without gradients
        with torch.no_grad():
            from gaussctrl_exp_amd.fused import render_fused
            render_fused(scene, cam, deg, bg)
        events.append(("phase forward", t0, clock()))
        return t0
    tr.zero_grad()
    t1 = clock()
    out = tr._render(cam, bg, gt=gt)
    t2 = clock()
    if out.get("backward") is not None:  # the direct fused step (fused._DirectCtx)
        out["backward"]()
    else:
        loss = out["loss"]
        seed = getattr(tr, "_seed", None)
        if seed is None:
            seed = tr._seed = torch.ones_like(loss)
        loss.backward(seed)
    t3 = clock()
    events.append(("phase zero_grad", t0, t1))
    events.append(("phase forward", t1, t2))
    events.append(("phase backward", t2, t3))
    return t0


for _ in range(20):
    step()
torch.cuda.synchronize()
acc = collections.defaultdict(lambda: [0.0, 0.0, 0])
spans = []
for s in range(steps):
    events.clear()
    if s == 0:
        small.clear()
    t0 = step()
    t_end = clock()
    spans.append(t_end - t0)
    seen = collections.Counter()
    for name, a, b in events:
        k = seen[name]
        seen[name] += 1
        e = acc[(name, k)]
        e[0] += a - t0
        e[1] += b - a
        e[2] += 1
torch.cuda.synchronize()
for label, (c, t) in sorted(small.items()):
    print(f"  {label}: {c / steps:.1f} calls, {1e6 * t / steps:.1f} us per step")
print(f"{cfg}: host time per step (no sync between steps) {1e6 * sum(spans) / len(spans):.1f} us")
rows = sorted(acc.items(), key=lambda kv: kv[1][0] / kv[1][2])
for (name, k), (start, dur, c) in rows:
    print(f"  +{1e6 * start / c:8.1f} us  {1e6 * dur / c:8.1f} us  {name}{' #%d' % k if k else ''}")
# the same loop, synchronised per step: the device-bound lower bound of the host path
t0 = clock()
for _ in range(50):
    step()
    torch.cuda.synchronize()
print(f"synchronised per step: {1e6 * (clock() - t0) / 50:.1f} us")
t0 = clock()
for _ in range(50):
    step()
torch.cuda.synchronize()
print(f"free-running: {1e6 * (clock() - t0) / 50:.1f} us per step")
