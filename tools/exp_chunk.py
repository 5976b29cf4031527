"""List-split backward: raster forward/backward time vs the chunk size, through the autograd
wrapper (clearing forward + record backward with its split plan), on one config (CFG env;
CHUNKS env: comma-separated chunk sizes, -1 = off, 0 = auto; FLAGS env: comma-separated
gsplat_debug_set_raster_variant flag words, each swept over CHUNKS)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
# the gsplat_debug_* switches live in the test library (include/gsplat_mi355x.h "test hooks")
os.environ.setdefault("GSPLAT_MI355X_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                        "..", "gaussctrl_exp_amd",
                                                        "libgsplat_mi355x_hooks.so"))
import bench  # noqa: E402
from gaussctrl_exp_amd import _lib, timing  # noqa: E402
from gaussctrl_exp_amd.project_gaussians import project_gaussians  # noqa: E402
from gaussctrl_exp_amd.rasterize import rasterize_gaussians  # noqa: E402

cfg = os.environ.get("CFG", "headline")
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
N, H, W = sc.num_points, cam.height, cam.width
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
colors = torch.rand(N, 3, device=dev)
opac = torch.sigmoid(sc.opacities).contiguous()
bg = torch.zeros(3, device=dev)
v_out = torch.randn(H, W, 3, device=dev)


def step():
    xy = xys.clone().requires_grad_()
    img = rasterize_gaussians(xy, depths, radii, conics, nth, colors, opac, H, W, bg)
    img.backward(v_out)
    return xy.grad


auto = None
res = {}
chunks = [int(c) for c in os.environ.get("CHUNKS", "-1,0,64,128,256,512,1024").split(",")]
flags = [int(f, 0) for f in os.environ.get("FLAGS", "0").split(",")]
for fl, ch in [(f, c) for f in flags for c in chunks]:
    _lib.call("gsplat_debug_set_raster_variant", 1, 0, fl)
    _lib.call("gsplat_debug_set_chunk", ch)
    for _ in range(3):
        g = step()
    if (fl, ch) == (flags[0], chunks[0]):
        ref = g.clone()
    else:
        err = (g - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-3, (ch, err)
    fw, bw = [], []
    for _ in range(5):
        with timing.timed_calls() as tm:
            for _ in range(5):
                step()
            s = tm.summary()
        fw.append(sum(v[1] for k, v in s.items() if "rasterize_forward" in k))
        bw.append(sum(v[1] for k, v in s.items() if "rasterize_backward" in k or
                      "grad_records_split" in k))
    res[fl, ch] = (np.median(fw), np.median(bw))
_lib.call("gsplat_debug_set_chunk", 0)
_lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)
print(f"{cfg}: N={N} image {W}x{H} auto chunk ="
      f" {_lib.query('gsplat_rasterize_chunk_size', cam.tile_bounds[0], cam.tile_bounds[1], 10**6)}"
      " (per 1M intersections)")
for (fl, ch), (f, b) in res.items():
    lbl = {-1: "off", 0: "auto"}.get(ch, str(ch))
    print(f"  flags {fl:#x} chunk {lbl:>5s}: fwd {f:.3f} ms  bwd {b:.3f} ms  sum {f + b:.3f}")
