"""Attribution of the record backward's time, on the bench step of CFG.

Run with the attribution library (tools/bwd_attr.sh: GSPLAT_MI355X_LIB=ab/libattr.so, built
with -DGS_BWD_ATTR) the strip backward logs per wave, in s_memtime cycles, its life, its
prologue (pixel loads up to the first staged round), the time inside its blend rounds and,
within those, the reduce9 + record-atomic tails of the iterations that had a valid pair.  Then
  staging   = life - prologue - blend     (id -> record gathers, keep-bit walk, LDS syncs)
  tail      = the reduce9 + atomic part of the blend rounds
  blend     = blend - tail                (the per-pixel math of the iterations)
and, from the wave start / end times (s_memrealtime, 100 MHz), the end-of-launch imbalance:
the span from the 90th-percentile wave end to the last one, and the mean share of the
launch's SIMD slots that are idle while waves are still running.  The record backward's time
per call with this library and with the shipped one (TIME_ONLY=1 under the shipped library)
shows what the timers cost."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from gaussctrl_exp_amd import _lib, timing  # noqa: E402
from gaussctrl_exp_amd.train import TrainStep  # noqa: E402

cfg = os.environ.get("CFG", "headline")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
scene, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
H, W = cam.height, cam.width
deg = bench.CONFIGS[cfg][3]
gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(1000)).to(dev)
bg = torch.zeros(3, device=dev)
t = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")


def step():
    t.zero_grad()
    t.forward_backward(cam, gt, bg)


for _ in range(5):
    step()
torch.cuda.synchronize()
ENTRY = "gsplat_rasterize_backward_records_l1"
with timing.timed_calls() as tm:
    for _ in range(20):
        step()
    per = tm.summary()
bwd_ms = per[ENTRY][1] if ENTRY in per else None
lib = os.environ.get("GSPLAT_MI355X_LIB", "shipped")
out = {"config": cfg, "library": lib, "record_backward_ms": round(bwd_ms, 4) if bwd_ms else None}
if os.environ.get("TIME_ONLY"):
    print(json.dumps(out), flush=True)
    sys.exit(0)

tb = cam.tile_bounds
F = 11
cap = 16 * tb[0] * tb[1] * 4  # > waves of any backward geometry / item list
log = torch.zeros(cap * F, dtype=torch.int64, device=dev)
_lib.call("gsplat_debug_wave_log", _lib.ptr(log))
try:
    step()
    torch.cuda.synchronize()
finally:
    _lib.call("gsplat_debug_wave_log", None)
a = log.view(cap, F).cpu().numpy().astype(np.float64)
a = a[a[:, 10] > 0]  # waves of the strip backward (life > 0)
t0, t1 = a[:, 0], a[:, 1]
life, pro, blend, tail = a[:, 10], a[:, 7], a[:, 5], a[:, 6]
rounds = (a[:, 8].astype(np.int64) >> 32).astype(np.float64)
iters = (a[:, 8].astype(np.int64) & 0xFFFFFFFF).astype(np.float64)
tail_it = a[:, 9]
tot = life.sum()
staging = life - pro - blend
span = (t1.max() - t0.min()) * 10.0  # ns (100 MHz)
# SIMD-slot occupancy over the launch: waves alive at each 100 ns
grid = np.arange(t0.min(), t1.max() + 1, 10)
alive = np.searchsorted(np.sort(t0), grid, side="right") - np.searchsorted(np.sort(t1), grid,
                                                                          side="right")
peak = alive.max()
p90 = np.percentile(t1, 90)
out.update({
    "waves": int(a.shape[0]),
    "kernel_span_us": round(span / 1e3, 2),
    "wave_life_us_mean": round(float((t1 - t0).mean()) * 10.0 / 1e3, 2),
    "cycles_per_ns": round(float(tot / ((t1 - t0).sum() * 10.0)), 3),
    "share_of_wave_time": {
        "prologue (pixel loads, keep-bit setup)": round(float(pro.sum() / tot), 4),
        "staging (id -> record gathers, walk, LDS syncs)": round(float(staging.sum() / tot), 4),
        "blend math (valid and invalid pairs)": round(float((blend - tail).sum() / tot), 4),
        "reduce9 + atomic tail": round(float(tail.sum() / tot), 4),
    },
    "rounds_per_wave": round(float(rounds.mean()), 2),
    "iterations_per_wave": round(float(iters.mean()), 2),
    "tail_iterations_frac": round(float(tail_it.sum() / max(iters.sum(), 1)), 4),
    "cycles_per_iteration": {
        "blend": round(float(blend.sum() / max(iters.sum(), 1)), 1),
        "staging per round": round(float(staging.sum() / max(rounds.sum(), 1)), 1),
        "tail per tail iteration": round(float(tail.sum() / max(tail_it.sum(), 1)), 1),
    },
    "imbalance": {
        "last_10pct_of_waves_end_span_us": round(float(t1.max() - p90) * 10.0 / 1e3, 2),
        "share_of_span_after_p90_end": round(float((t1.max() - p90) * 10.0 / span), 4),
        "peak_resident_waves": int(peak),
        "mean_resident_over_peak": round(float(alive.mean() / peak), 4),
        "wave_life_max_over_mean": round(float((t1 - t0).max() / (t1 - t0).mean()), 2),
    },
})
print(json.dumps(out), flush=True)
