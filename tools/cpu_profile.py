"""Host-side cost of one bench step: torch.profiler CPU self-time per op and the wall time
of the step's Python code vs GPU time (is the step launch-bound?)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench
from gaussctrl_exp_amd.scene import synthetic_scene
from gaussctrl_exp_amd.train import TrainStep

cfg = os.environ.get("CFG", "headline")
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
scene, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
H, W = cam.height, cam.width
gt = torch.rand(H, W, 3, device=dev)
bg = torch.zeros(3, device=dev)
tr = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1",
               render_mode=os.environ.get("RENDER", "fused"))


def step():
    tr.zero_grad()
    tr.forward_backward(cam, gt, bg)


for _ in range(5):
    step()
torch.cuda.synchronize()
# host time of the step's Python with the GPU kept busy, and the synced wall time
t0 = time.perf_counter(); step(); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
print(f"python step call {1e3*(t1-t0):.3f} ms, until GPU idle {1e3*(t2-t0):.3f} ms")
for _ in range(15):
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    print(f"10 steps {1e2*(time.perf_counter()-t0):.3f} ms/step", flush=True)
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU]) as prof:
    for _ in range(5):
        step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))
import cProfile
import pstats
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
