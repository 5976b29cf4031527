"""Why compute_sh_forward takes ~65 us per call in the unchanged-caller leg at the headline when
the same kernel streams 1M Gaussians' coefficients in ~35-39 us on its own
(profiles/r06_sh_stream_bench.txt): the drop-in spherical_harmonics timed with HIP events
(a) on a resident coefficient tensor, (b) right behind the caller's torch.cat that writes it,
(c) the cat alone, (d) cat + SH inside the caller's whole step (scene.render).  Run on the GPU."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
from gaussctrl_exp_amd.sh import spherical_harmonics

dev = torch.device("cuda:0")
scene, cam = bench.make_workload("headline", 0, dev)
cam = cam.to(dev)
reps = 30


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


with torch.no_grad():
    coeffs = torch.cat((scene.features_dc[:, None, :], scene.features_rest), dim=1)
    vd = scene.means - cam.c2w[..., :3, 3]
    vd = vd / vd.norm(dim=-1, keepdim=True)
    t_sh = timed(lambda: spherical_harmonics(3, vd, coeffs))
    t_cat = timed(lambda: torch.cat((scene.features_dc[:, None, :], scene.features_rest), dim=1))
    t_both = timed(lambda: spherical_harmonics(
        3, vd, torch.cat((scene.features_dc[:, None, :], scene.features_rest), dim=1)))
print(f"sh on resident coeffs      {t_sh:7.1f} us")
print(f"cat alone                  {t_cat:7.1f} us")
print(f"cat then sh                {t_both:7.1f} us  (sh part ~{t_both - t_cat:.1f} us)")
sys.stdout.flush()
