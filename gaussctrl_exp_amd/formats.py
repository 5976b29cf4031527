"""On-disk formats of the reference: nerfstudio transforms.json cameras,
the ASCII sparse_pc.ply seed point cloud, and splatfacto checkpoints.  Nothing here is on
the per-step hot path: the loaders produce the GCCamera / GaussianScene objects the hot path
consumes, so the real-scene configurations (C3 bear, C4 garden) run without nerfstudio.

* `load_transforms` follows GaussCtrlDataParser._generate_dataparser_outputs
  (/root/reference/gaussctrl/gc_dataparser_ns.py:106-330):
  - frames are sorted by file name (:145-151);
  - intrinsics come from the file or per frame (:122-176);
  - poses are oriented and centred by nerfstudio's auto_orient_and_center_poses (:254-259,
    orientation "up", centre "poses" by default) and scaled so that the largest |t| is 1
    (:261-267);
  - the intrinsics are divided by the downscale factor (:316-317).
  nerfstudio itself (1.0.0, `cameras/camera_utils.py`) is not installed here.  Its
  rotation_matrix_between / auto_orient_and_center_poses are restated below from the
  published algorithm, so parity with nerfstudio's own output is unpinned.  The tests check
  the defining properties instead: mean up-vector -> +z, mean origin -> 0, max |t| -> 1,
  proper rotations.
* `load_points` is _load_3D_points (:436-471): the same transform and scale applied to
  sparse_pc.ply.  When transforms.json carries "applied_scale", the points use the scale
  multiplied by it (:341-343), as the reference does.
* `load_splatfacto_ckpt` / `save_splatfacto_ckpt`: the checkpoint dict written at
  gc_trainer.py:156-168 ({"step", "pipeline": state_dict, ...}), read with
  torch.load(weights_only=True).  The Gaussian parameters sit under
  "_model.gauss_params.<name>" (nerfstudio 1.0 splatfacto) or "_model.<name>" (0.3.x).
  Lens distortion (k1, k2, p1, p2 of OPENCV cameras) is parsed but, as in splatfacto's
  gsplat render, not applied.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from .camera import GCCamera, gc_camera
from .scene import PARAM_NAMES, GaussianScene, read_ply_points

MAX_AUTO_RESOLUTION = 1600  # gc_dataparser_ns.py:47


def rotation_matrix_between(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Rotation taking direction a onto direction b (Rodrigues; nerfstudio camera_utils)."""
    a = a / torch.linalg.norm(a)
    b = b / torch.linalg.norm(b)
    v = torch.linalg.cross(a, b)
    eps = 1e-6
    if torch.sum(torch.abs(v)) < eps:  # a and b (anti-)parallel: any perpendicular axis
        x = torch.tensor([1.0, 0.0, 0.0]) if abs(a[0]) < eps else torch.tensor([0.0, 1.0, 0.0])
        v = torch.linalg.cross(a, x.to(a.dtype))
    v = v / torch.linalg.norm(v)
    skew = torch.tensor([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]],
                        dtype=a.dtype)
    theta = torch.acos(torch.clip(torch.dot(a, b), -1, 1))
    return torch.eye(3, dtype=a.dtype) + torch.sin(theta) * skew + \
        (1 - torch.cos(theta)) * (skew @ skew)


def auto_orient_and_center_poses(poses: torch.Tensor, method: str = "up",
                                 center_method: str = "poses"):
    """poses [N,4,4] (or [N,3,4]) camera-to-world -> (oriented poses [N,3,4], transform
    [3,4]), nerfstudio's orientation methods "up", "pca", "none" and centre methods
    "poses", "none"."""
    if poses.shape[-2] == 3:
        bottom = torch.tensor([0.0, 0.0, 0.0, 1.0], dtype=poses.dtype).expand(
            poses.shape[0], 1, 4)
        poses = torch.cat([poses, bottom], dim=-2)
    origins = poses[..., :3, 3]
    mean_origin = torch.mean(origins, dim=0)
    if center_method == "poses":
        translation = mean_origin
    elif center_method == "none":
        translation = torch.zeros_like(mean_origin)
    else:
        raise NotImplementedError(f"center_method {center_method!r} (poses, none supported)")
    if method == "up":
        up = torch.mean(poses[:, :3, 1], dim=0)
        up = up / torch.linalg.norm(up)
        rotation = rotation_matrix_between(up, torch.tensor([0.0, 0.0, 1.0], dtype=up.dtype))
        transform = torch.cat([rotation, rotation @ -translation[..., None]], dim=-1)
        oriented = transform @ poses
    elif method == "pca":
        diff = origins - mean_origin
        _, eigvec = torch.linalg.eigh(diff.T @ diff)
        eigvec = torch.flip(eigvec, dims=(-1,))
        if torch.linalg.det(eigvec) < 0:
            eigvec[:, 2] = -eigvec[:, 2]
        transform = torch.cat([eigvec, eigvec @ -translation[..., None]], dim=-1)
        oriented = transform @ poses
        if oriented.mean(dim=0)[2, 1] < 0:
            oriented[:, 1:3] = -1 * oriented[:, 1:3]
            transform[1:3, :] = -1 * transform[1:3, :]
    elif method == "none":
        transform = torch.eye(4, dtype=poses.dtype)
        transform[:3, 3] = -translation
        transform = transform[:3, :]
        oriented = transform @ poses
    else:
        raise NotImplementedError(f"orientation method {method!r} (up, pca, none supported)")
    return oriented, transform


@dataclass
class TransformsData:
    """What the dataparser hands the pipeline, for the hot path's purposes."""
    cameras: List[GCCamera]
    image_paths: List[str]
    transform_matrix: torch.Tensor  # [3,4] saved -> dataparser coordinates
    scale_factor: float             # applied to pose translations
    points_scale: float             # applied to sparse_pc.ply points (x applied_scale)
    ply_path: Optional[str]
    distortion: Dict[str, float] = field(default_factory=dict)


def load_transforms(path: str, downscale_factor: Optional[int] = None,
                    orientation_method: str = "up", center_method: str = "poses",
                    auto_scale_poses: bool = True, scale_factor: float = 1.0,
                    device="cpu") -> TransformsData:
    """nerfstudio transforms.json (a file, or a directory holding one) -> cameras in the
    reference's dataparser coordinates (gc_dataparser_ns.py:106-330; train split with the
    default train_split_fraction 1.0, i.e. every frame)."""
    if os.path.isdir(path):
        data_dir, path = path, os.path.join(path, "transforms.json")
    else:
        data_dir = os.path.dirname(path)
    with open(path) as f:
        meta = json.load(f)
    frames = sorted(meta["frames"], key=lambda fr: os.path.basename(fr["file_path"]))

    def intr(key, frame, cast):
        if key in meta:
            return cast(meta[key])
        if key not in frame:
            raise ValueError(f"{path}: {key} given neither globally nor per frame")
        return cast(frame[key])

    if downscale_factor is None:  # auto (:484-498): only the image size is needed
        w0, h0 = intr("w", frames[0], int), intr("h", frames[0], int)
        df = 0
        while max(w0, h0) / 2 ** df > MAX_AUTO_RESOLUTION and os.path.isdir(
                os.path.join(data_dir, f"images_{2 ** (df + 1)}")):
            df += 1
        downscale_factor = 2 ** df
    poses = torch.tensor([fr["transform_matrix"] for fr in frames], dtype=torch.float32)
    method = meta.get("orientation_override", orientation_method)
    poses, transform = auto_orient_and_center_poses(poses, method, center_method)
    scale = 1.0
    if auto_scale_poses:
        scale /= float(torch.max(torch.abs(poses[:, :3, 3])))
    scale *= scale_factor
    poses[:, :3, 3] *= scale
    points_scale = scale * float(meta.get("applied_scale", 1.0))
    s = 1.0 / downscale_factor
    cams, paths = [], []
    for fr, c2w in zip(frames, poses):
        fx, fy = intr("fl_x", fr, float) * s, intr("fl_y", fr, float) * s
        cx, cy = intr("cx", fr, float) * s, intr("cy", fr, float) * s
        W, H = int(intr("w", fr, int) * s), int(intr("h", fr, int) * s)
        cams.append(gc_camera(c2w[:3, :4], fx, fy, cx, cy, W, H, device=device))
        paths.append(os.path.join(data_dir, fr["file_path"]))
    dist = {k: float(meta[k]) for k in ("k1", "k2", "k3", "k4", "p1", "p2") if k in meta}
    ply = meta.get("ply_file_path")
    return TransformsData(cams, paths, transform, scale, points_scale,
                          os.path.join(data_dir, ply) if ply else None, dist)


def transform_points(xyz: torch.Tensor, transform_matrix: torch.Tensor, scale: float):
    """File-coordinate points [M,3] -> dataparser coordinates (gc_dataparser_ns.py:455-466)."""
    xyz_h = torch.cat([xyz, torch.ones_like(xyz[..., :1])], -1)
    return (xyz_h @ transform_matrix.to(xyz.dtype).T) * scale


def load_points(ply_path: str, transform_matrix: torch.Tensor, scale: float):
    """sparse_pc.ply -> (xyz [M,3] in dataparser coordinates, rgb uint8 [M,3] or None)."""
    xyz, rgb = read_ply_points(ply_path)
    return transform_points(xyz, transform_matrix, scale), rgb


def rescale_cameras(cams: List[GCCamera], factor: float) -> List[GCCamera]:
    """nerfstudio Cameras.rescale_output_resolution: intrinsics and image size x factor."""
    return [gc_camera(c.c2w, c.fx * factor, c.fy * factor, c.cx * factor, c.cy * factor,
                      int(c.width * factor), int(c.height * factor), device=c.c2w.device)
            for c in cams]


_PREFIXES = ("_model.gauss_params.", "_model.")


def load_splatfacto_ckpt(path: str, device="cpu") -> GaussianScene:
    """Gaussian parameters of a splatfacto / GaussCtrl checkpoint (gc_trainer.py:156-168),
    loaded with torch.load(weights_only=True) -- nothing in the file is executed."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    state = ckpt.get("pipeline", ckpt)
    params = {}
    for name in PARAM_NAMES:
        for pre in _PREFIXES:
            if pre + name in state:
                params[name] = state[pre + name]
                break
        else:
            raise KeyError(f"{path}: no '{name}' Gaussian parameter (looked for "
                           f"{[p + name for p in _PREFIXES]})")
    n = params["means"].shape[0]
    if any(v.shape[0] != n for v in params.values()):
        raise ValueError(f"{path}: Gaussian parameter tensors disagree on N")
    rest = params["features_rest"]
    k = rest.shape[1] + 1
    if rest.dim() != 3 or rest.shape[2] != 3 or int(math.isqrt(k)) ** 2 != k:
        raise ValueError(f"{path}: features_rest must be [N, (d+1)^2 - 1, 3]")
    return GaussianScene(*[params[nm].float().contiguous().to(device) for nm in PARAM_NAMES])


def save_splatfacto_ckpt(scene: GaussianScene, path: str, step: int = 0):
    """Write the parameters in the nerfstudio 1.0 layout read by load_splatfacto_ckpt."""
    state = {f"_model.gauss_params.{nm}": getattr(scene, nm).detach().cpu()
             for nm in PARAM_NAMES}
    torch.save({"step": int(step), "pipeline": state}, path)
