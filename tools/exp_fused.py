"""Timing of the fused preprocess kernels against their unfused counterparts on the headline
scene (HIP events on the launch stream, median of 5 rounds of 20 calls; one process)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.scene import synthetic_scene

dev = torch.device("cuda:0")
cfg = os.environ.get("CFG", "headline")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
N, H, W = sc.num_points, cam.height, cam.width
tb = cam.tile_bounds
P, st = _lib.ptr, _lib.stream(dev)
f = lambda *s: torch.empty(*s, device=dev)
xys, depths, conics, colors, opac = f(N, 2), f(N), f(N, 3), f(N, 3), f(N)
radii = torch.empty(N, device=dev, dtype=torch.int32)
nth = torch.empty(N, device=dev, dtype=torch.int32)
rec = torch.empty(N * 64, device=dev, dtype=torch.uint8)
campos = cam.c2w[:3, 3].contiguous()
sc1 = synthetic_scene(N, 0, seed=10, scale_lo=0.005, scale_hi=0.02, device=dev)


def fused_fwd(s=sc, records=True):
    K = s.features_rest.shape[1] + 1
    _lib.call("gsplat_fused_preprocess_forward", N, K, {1: 0, 16: 3}[K],
              P(s.means), P(s.scales), P(s.quats), P(s.opacities), P(s.features_dc),
              P(s.features_rest) if K > 1 else None, P(cam.viewmat), P(cam.projmat), P(campos),
              cam.fx, cam.fy, cam.cx, cam.cy, H, W, tb[0], tb[1], 0.01, P(xys), P(depths),
              P(radii), P(conics), P(nth), P(colors), P(opac), P(rec) if records else None, None,
              None, st)


fused_fwd()
v = [f(N, 3), f(N, 3), f(N, 4), f(N), f(N, 3), f(N, 15, 3)]


def fused_bwd():
    _lib.call("gsplat_fused_preprocess_backward", N, 16, 3, P(sc.means), P(sc.scales),
              P(sc.quats), P(cam.viewmat), P(cam.projmat), P(campos), cam.fx, cam.fy, cam.cx,
              cam.cy, H, W, P(radii), P(conics), P(colors), P(opac), P(rec), *[P(x) for x in v],
              None, st)


import ctypes
mv = [(torch.zeros_like(t), torch.zeros_like(t)) for t in
      (sc.means, sc.scales, sc.quats, sc.opacities, sc.features_dc, sc.features_rest)]
M = (ctypes.c_void_p * 6)(*[m.data_ptr() for m, _ in mv])
V = (ctypes.c_void_p * 6)(*[v.data_ptr() for _, v in mv])
LR = (ctypes.c_float * 6)(1e-9, 1e-9, 1e-9, 1e-9, 1e-9, 1e-9)  # keep the scene ~fixed
pc = [t.clone() for t in (sc.means, sc.scales, sc.quats, sc.opacities, sc.features_dc,
                          sc.features_rest)]


def fused_bwd_adam():
    _lib.call("gsplat_fused_preprocess_backward_adam", N, 16, 3, *[P(t) for t in pc],
              P(cam.viewmat), P(cam.projmat), P(campos), cam.fx, cam.fy, cam.cx, cam.cy, H, W,
              P(radii), P(conics), P(colors), P(opac), P(rec), ctypes.cast(M, ctypes.c_void_p),
              ctypes.cast(V, ctypes.c_void_p), ctypes.cast(LR, ctypes.c_void_p), 1, 0.9, 0.999,
              1e-15, st)


def adam_sep():
    Pp = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in pc])
    G = (ctypes.c_void_p * 6)(*[x.data_ptr() for x in v])
    n = (ctypes.c_int64 * 6)(*[t.numel() for t in pc])
    _lib.call("gsplat_adam_step", 6, ctypes.cast(Pp, ctypes.c_void_p),
              ctypes.cast(G, ctypes.c_void_p), ctypes.cast(M, ctypes.c_void_p),
              ctypes.cast(V, ctypes.c_void_p), ctypes.cast(n, ctypes.c_void_p),
              ctypes.cast(LR, ctypes.c_void_p), 1, 0.9, 0.999, 1e-15, st)


scales = torch.exp(sc.scales)
quats = sc.quats / sc.quats.norm(dim=-1, keepdim=True)
cov3d = f(N, 6)
coeffs = torch.cat([sc.features_dc[:, None], sc.features_rest], 1).contiguous()
vd = sc.means - campos
vd = (vd / vd.norm(dim=-1, keepdim=True)).contiguous()


def proj_fwd():
    _lib.call("gsplat_project_gaussians_forward", N, P(sc.means), P(scales), 1.0, P(quats),
              P(cam.viewmat), P(cam.projmat), cam.fx, cam.fy, cam.cx, cam.cy, H, W, tb[0], tb[1],
              0.01, P(cov3d), P(xys), P(depths), P(radii), P(conics), P(nth), st)


def sh_fwd():
    _lib.call("gsplat_compute_sh_forward", N, 3, 3, P(vd), P(coeffs), P(colors), st)


def timeit(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


cases = {"fused_fwd K16": fused_fwd, "fused_fwd K16 no records": lambda: fused_fwd(records=False),
         "fused_fwd K1 (projection + activations)": lambda: fused_fwd(sc1),
         "fused_bwd K16": fused_bwd, "fused_bwd+adam K16": fused_bwd_adam,
         "adam_step (separate)": adam_sep, "project_fwd": proj_fwd, "sh_fwd": sh_fwd}
res = {k: [] for k in cases}
for _ in range(5):
    for k, fn in cases.items():
        fn()
        torch.cuda.synchronize()
        res[k].append(timeit(fn))
print(f"{cfg}: N={N} lib={_lib.LIB_PATH}")
for k in cases:
    print(f"{k:45s} {np.median(res[k]):8.1f} us")
