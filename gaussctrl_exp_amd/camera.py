"""Camera conventions of the reference caller (gaussctrl/gc_model.py:117-155).

`gc_camera` turns a nerfstudio camera-to-world matrix (OpenGL axes: camera looks down -z,
y up) and pinhole intrinsics into exactly the argument tuple gc_model passes to
`project_gaussians`: viewmat [3,4] after the diag(1,-1,-1) axis flip (gc_model.py:131-138),
projmat = P @ viewmat with nerfstudio splatfacto's projection_matrix (znear 0.001, zfar
1000; identical to gaussctrl/ad_render.py:49-67), and tile_bounds (gc_model.py:151-155).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

BLOCK_X, BLOCK_Y = 16, 16


def projection_matrix(znear, zfar, fovx, fovy, device="cpu"):
    """splatfacto's OpenGL-style projection with NDC z in [0,1] (ad_render.py:49-67)."""
    t = znear * math.tan(0.5 * fovy)
    b = -t
    r = znear * math.tan(0.5 * fovx)
    l = -r
    n = znear
    f = zfar
    return torch.tensor(
        [[2 * n / (r - l), 0.0, (r + l) / (r - l), 0.0],
         [0.0, 2 * n / (t - b), (t + b) / (t - b), 0.0],
         [0.0, 0.0, (f + n) / (f - n), -1.0 * f * n / (f - n)],
         [0.0, 0.0, 1.0, 0.0]], device=device)


@dataclass
class GCCamera:
    viewmat: torch.Tensor  # [3,4] world -> camera (gsplat axes)
    projmat: torch.Tensor  # [4,4] = P @ viewmat4x4
    fx: float
    fy: float
    cx: float
    cy: float
    height: int
    width: int
    tile_bounds: tuple
    c2w: torch.Tensor      # [3,4] nerfstudio convention

    def project_args(self):
        """Positional args after (means, scales, glob_scale, quats) -- gc_model.py:179-187."""
        return (self.viewmat, self.projmat, self.fx, self.fy, self.cx, self.cy, self.height,
                self.width, self.tile_bounds)

    def to(self, device):
        return GCCamera(self.viewmat.to(device), self.projmat.to(device), self.fx, self.fy,
                        self.cx, self.cy, self.height, self.width, self.tile_bounds,
                        self.c2w.to(device))


def gc_camera(c2w, fx, fy, cx, cy, width, height, device="cpu") -> GCCamera:
    """Reproduces GaussCtrlModel.get_outputs' camera math (gc_model.py:117-155)."""
    c2w = torch.as_tensor(c2w, dtype=torch.float32, device=device)[:3, :4]
    R = c2w[:3, :3]
    T = c2w[:3, 3:4]
    R_edit = torch.diag(torch.tensor([1, -1, -1], device=device, dtype=R.dtype))
    R = R @ R_edit
    R_inv = R.T
    T_inv = -R_inv @ T
    viewmat = torch.eye(4, device=device, dtype=R.dtype)
    viewmat[:3, :3] = R_inv
    viewmat[:3, 3:4] = T_inv
    fovx = 2 * math.atan(width / (2 * fx))
    fovy = 2 * math.atan(height / (2 * fy))
    projmat = projection_matrix(0.001, 1000, fovx, fovy, device=device)
    tile_bounds = (int((width + BLOCK_X - 1) // BLOCK_X), int((height + BLOCK_Y - 1) // BLOCK_Y),
                   1)
    return GCCamera(viewmat[:3, :].contiguous(), (projmat @ viewmat).contiguous(), float(fx),
                    float(fy), float(cx), float(cy), int(height), int(width), tile_bounds, c2w)


def look_at_c2w(eye, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)):
    """nerfstudio/OpenGL camera-to-world [3,4] at `eye` looking at `target`."""
    eye = torch.tensor(eye, dtype=torch.float32)
    target = torch.tensor(target, dtype=torch.float32)
    up = torch.tensor(up, dtype=torch.float32)
    fwd = target - eye
    fwd = fwd / fwd.norm()
    right = torch.linalg.cross(fwd, up)
    if right.norm() < 1e-6:
        right = torch.linalg.cross(fwd, torch.tensor([0.0, 1.0, 0.0]))
    right = right / right.norm()
    cam_up = torch.linalg.cross(right, fwd)
    # OpenGL: x = right, y = up, z = -forward
    R = torch.stack([right, cam_up, -fwd], dim=1)
    return torch.cat([R, eye[:, None]], dim=1)


def synthetic_camera(width, height, fov_x_deg=50.0, eye=(0.0, 0.0, 4.0), device="cpu"):
    """SURVEY.md §8(d) synthetic camera: at (0,0,4) looking at the origin, fov_x 50 deg,
    fx = fy = 0.5*W/tan(25 deg), principal point at the image centre."""
    fx = 0.5 * width / math.tan(math.radians(fov_x_deg) / 2)
    c2w = look_at_c2w(eye, up=(0.0, 1.0, 0.0))
    return gc_camera(c2w, fx, fx, width / 2.0, height / 2.0, width, height, device=device)
