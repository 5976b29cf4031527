"""Eval render (gc_model.get_outputs with return_depth) at the headline size: the reference
caller's two rasterize calls (with and without the binning reuse) vs the fused RGB+depth pass, and
the fused preprocess + RGB+depth pass (fused.render_fused_eval)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gaussctrl_exp_amd import rasterize as R  # noqa: E402
from gaussctrl_exp_amd.camera import synthetic_camera  # noqa: E402
from gaussctrl_exp_amd.scene import render, synthetic_scene  # noqa: E402

dev = torch.device("cuda:0")
sc = synthetic_scene(1_000_000, 3, seed=10, device=dev)
cam = synthetic_camera(1080, 1080).to(dev)
bg = torch.zeros(3, device=dev)


class NoCache(R._BinCache):
    def get(self, *a):
        return None


def run(label, fused, cache=True, reps=30):
    R._BIN_CACHE = R._BinCache() if cache else NoCache()
    with torch.no_grad():
        for _ in range(5):
            render(sc, cam, 3, bg, return_depth=True, fused_depth=fused)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            render(sc, cam, 3, bg, return_depth=True, fused_depth=fused)
        torch.cuda.synchronize()
    print(f"{label}: {(time.perf_counter() - t) / reps * 1e3:.3f} ms per eval render")


run("two rasterize calls, no binning reuse", False, cache=False)
run("two rasterize calls, binning reused", False)
run("fused RGB+depth pass", True)


def run_fused_eval(reps=30):
    from gaussctrl_exp_amd.fused import render_fused_eval
    for _ in range(5):
        render_fused_eval(sc, cam, 3, bg)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        render_fused_eval(sc, cam, 3, bg)
    torch.cuda.synchronize()
    print(f"fused preprocess + RGB+depth pass (render_fused_eval): "
          f"{(time.perf_counter() - t) / reps * 1e3:.3f} ms per eval render")


run_fused_eval()
