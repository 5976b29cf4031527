"""Gaussian scenes and the reference caller's render step.

`render` is GaussCtrlModel.get_outputs' hot path (gaussctrl/gc_model.py:158-238) with the
nerfstudio Camera/Model plumbing removed: the same activations (exp scales, normalised
quats, concatenated SH coefficients, sigmoid opacities), the same calls into the gsplat
API, in the same order, with the same arguments.  `synthetic_scene` draws the random
scenes of SURVEY.md §8(d); `scene_from_ply` seeds Gaussians around a reference point cloud
(data/*/sparse_pc.ply).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from .camera import GCCamera
from .project_gaussians import project_gaussians
from .rasterize import rasterize_gaussians, rasterize_gaussians_rgbd
from .sh import num_sh_bases, spherical_harmonics

PARAM_NAMES = ("means", "scales", "quats", "opacities", "features_dc", "features_rest")
PARAM_WIDTH = {"means": 3, "scales": 3, "quats": 4, "opacities": 1, "features_dc": 3}


@dataclass
class GaussianScene:
    """splatfacto parameter layout (gc_model.py:158-170): raw (pre-activation) tensors."""
    means: torch.Tensor          # [N,3]
    scales: torch.Tensor         # [N,3] log-scales
    quats: torch.Tensor          # [N,4] unnormalised (w,x,y,z)
    opacities: torch.Tensor      # [N,1] logits
    features_dc: torch.Tensor    # [N,3]
    features_rest: torch.Tensor  # [N,K-1,3]

    @property
    def num_points(self) -> int:
        return self.means.shape[0]

    def params(self):
        return [getattr(self, k) for k in PARAM_NAMES]

    def to(self, device):
        return GaussianScene(*[p.to(device) for p in self.params()])

    def requires_grad_(self, flag=True):
        for p in self.params():
            p.requires_grad_(flag)
        return self

    def detach(self):
        return GaussianScene(*[p.detach() for p in self.params()])


def synthetic_scene(n: int, sh_degree: int = 3, seed: int = 0, scale_lo: float = 0.005,
                    scale_hi: float = 0.03, extent: float = 1.5, opacity_lo: float = -2.0,
                    opacity_hi: float = 3.0, device="cpu") -> GaussianScene:
    """means ~ U([-e,e]^3), log-scales = log U(lo,hi), quats ~ N(0,1)^4,
    opacity logits ~ U(-2,3), dc ~ N(0,0.5), rest ~ N(0,0.05); drawn on a CPU generator so
    every device sees the same scene."""
    g = torch.Generator().manual_seed(seed)
    K = num_sh_bases(sh_degree)
    means = (torch.rand(n, 3, generator=g) * 2 - 1) * extent
    scales = torch.log(torch.rand(n, 3, generator=g) * (scale_hi - scale_lo) + scale_lo)
    quats = torch.randn(n, 4, generator=g)
    opac = torch.rand(n, 1, generator=g) * (opacity_hi - opacity_lo) + opacity_lo
    dc = torch.randn(n, 3, generator=g) * 0.5
    rest = torch.randn(n, K - 1, 3, generator=g) * 0.05
    return GaussianScene(means, scales, quats, opac, dc, rest).to(device)


def read_ply_points(path: str):
    """ASCII PLY vertices (x y z [r g b]) as (xyz float32 [M,3], rgb uint8 [M,3] or None)."""
    with open(path, "rb") as f:
        header = []
        while True:
            line = f.readline().decode("ascii", errors="replace").strip()
            header.append(line)
            if line == "end_header":
                break
        nvert = 0
        props = []
        for h in header:
            if h.startswith("element vertex"):
                nvert = int(h.split()[-1])
            elif h.startswith("property"):
                props.append(h.split()[-1])
        if "format ascii" not in " ".join(header):
            raise ValueError(f"{path}: only ASCII PLY is supported")
        import numpy as np
        data = np.loadtxt(f, max_rows=nvert, dtype=np.float64, ndmin=2)
    xyz = data[:, [props.index("x"), props.index("y"), props.index("z")]].astype("float32")
    rgb = None
    if all(c in props for c in ("red", "green", "blue")):
        rgb = data[:, [props.index("red"), props.index("green"),
                       props.index("blue")]].astype("uint8")
    return torch.from_numpy(xyz), (torch.from_numpy(rgb) if rgb is not None else None)


def scene_from_points(xyz: torch.Tensor, rgb: Optional[torch.Tensor], n: int,
                      sh_degree: int = 3, seed: int = 0, jitter: float = 0.02,
                      scale_lo: float = 0.005, scale_hi: float = 0.03,
                      device="cpu") -> GaussianScene:
    """n Gaussians seeded around a point cloud (copies of the points + N(0, jitter) offsets),
    DC colour from the point colour (splatfacto's RGB2SH init), other params as
    synthetic_scene."""
    g = torch.Generator().manual_seed(seed)
    m = xyz.shape[0]
    idx = torch.randint(0, m, (n,), generator=g)
    means = xyz[idx] + torch.randn(n, 3, generator=g) * jitter
    base = synthetic_scene(n, sh_degree, seed=seed + 1, scale_lo=scale_lo, scale_hi=scale_hi)
    dc = base.features_dc
    if rgb is not None:
        dc = (rgb[idx].float() / 255.0 - 0.5) / 0.28209479177387814
    return GaussianScene(means, base.scales, base.quats, base.opacities, dc,
                         base.features_rest).to(device)


def render(scene: GaussianScene, cam: GCCamera, sh_degree_to_use: int, background: torch.Tensor,
           return_depth: bool = False, api=None, fused_depth: bool = False):
    """GaussCtrlModel.get_outputs' hot path (gc_model.py:158-238) on a GCCamera.

    `api` swaps the gsplat implementation (tests pass the CPU-oracle emulation); by default
    the MI355X kernels are used.  With return_depth, the depth image comes from a second
    rasterize call as in gc_model.py:225-236, or -- fused_depth=True, MI355X kernels, no
    autograd -- from the single fused RGB+depth pass (rasterize_gaussians_rgbd).  Returns dict(rgb [H,W,3], accumulation [H,W,1],
    depth [H,W,1] or None, xys, radii)."""
    project = api.project_gaussians if api is not None else project_gaussians
    sh_eval = api.spherical_harmonics if api is not None else spherical_harmonics
    raster = api.rasterize_gaussians if api is not None else rasterize_gaussians
    colors_crop = torch.cat((scene.features_dc[:, None, :], scene.features_rest), dim=1)
    quats = scene.quats
    xys, depths, radii, conics, num_tiles_hit, cov3d = project(
        scene.means, torch.exp(scene.scales), 1, quats / quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    if radii.sum() == 0:
        rgb = background.repeat(cam.height, cam.width, 1)
        return {"rgb": rgb, "accumulation": None, "depth": None, "xys": xys, "radii": radii}
    if xys.requires_grad:
        xys.retain_grad()
    if colors_crop.shape[1] > 1:
        viewdirs = scene.means.detach() - cam.c2w.detach()[..., :3, 3]
        viewdirs = viewdirs / viewdirs.norm(dim=-1, keepdim=True)
        rgbs = sh_eval(sh_degree_to_use, viewdirs, colors_crop)
        rgbs = torch.clamp(rgbs + 0.5, min=0.0)
    else:
        rgbs = torch.sigmoid(colors_crop[:, 0, :])
    if return_depth and fused_depth:
        if api is not None:
            raise ValueError("fused_depth renders with the MI355X kernels only")
        rgb, depth_im, alpha = rasterize_gaussians_rgbd(
            xys, depths, radii, conics, num_tiles_hit, rgbs, torch.sigmoid(scene.opacities),
            cam.height, cam.width, background=background)
        alpha = alpha[..., None]
        rgb = torch.clamp(rgb, max=1.0)
        depth_im[alpha > 0] = depth_im[alpha > 0] / alpha[alpha > 0]
        depth_im[alpha == 0] = 1000
        return {"rgb": rgb, "depth": depth_im, "accumulation": alpha, "xys": xys, "radii": radii}
    rgb, alpha = raster(xys, depths, radii, conics, num_tiles_hit, rgbs,
                                     torch.sigmoid(scene.opacities), cam.height, cam.width,
                                     background=background, return_alpha=True)
    alpha = alpha[..., None]
    rgb = torch.clamp(rgb, max=1.0)
    depth_im = None
    if return_depth:
        depth_im = raster(xys, depths, radii, conics, num_tiles_hit,
                                       depths[:, None].repeat(1, 3),
                                       torch.sigmoid(scene.opacities), cam.height, cam.width,
                                       background=torch.zeros(3, device=xys.device))[..., 0:1]
        depth_im = depth_im.clone()
        depth_im[alpha > 0] = depth_im[alpha > 0] / alpha[alpha > 0]
        depth_im[alpha == 0] = 1000
    return {"rgb": rgb, "depth": depth_im, "accumulation": alpha, "xys": xys, "radii": radii}
