"""Same-process A/B of binning switches on the whole bench step (bench.py's fused fwd+bwd
step on CFG, default headline): ms per step for each setting, interleaved over REPS rounds so
box drift hits every setting alike.  Settings: bins_from_sort (tile table from the last tile
pass vs a bin-edges kernel), compact (depth sort drops culled keys), emit_pass0 (0 / 1 auto)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.train import TrainStep

cfg = os.environ.get("CFG", "headline")
reps = int(os.environ.get("REPS", "3"))
steps = int(os.environ.get("STEPS", "40"))
dev = torch.device("cuda:0")
N, W, H, deg, *_ = bench.CONFIGS[cfg]
scene, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(1000)).to(dev)
bg = torch.zeros(3, device=dev)
tr = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")
L = _lib.lib()


def step():
    tr.zero_grad()
    tr.forward_backward(cam, gt, bg)


SETTINGS = {
    "shipped": dict(bfs=1, compact=1, gen=1),
    "bin_edges": dict(bfs=0, compact=1, gen=1),
    "no_compact": dict(bfs=1, compact=0, gen=1),
}


def apply(s):
    _lib.call("gsplat_debug_bins_from_sort", s["bfs"])
    L.gsplat_debug_compact_depth_sort(s["compact"])
    L.gsplat_debug_emit_pass0(s["gen"])


res = {k: [] for k in SETTINGS}
for r in range(reps):
    for name, s in SETTINGS.items():
        apply(s)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / steps)
        print(f"{cfg} rep {r} {name}: {res[name][-1]:.4f} ms/step", flush=True)
apply(SETTINGS["shipped"])
for name, v in res.items():
    print(f"{cfg} {name}: min {min(v):.4f} median {sorted(v)[len(v) // 2]:.4f} ms/step")
