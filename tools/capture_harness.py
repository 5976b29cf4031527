"""Capture golden harness vectors from the REFERENCE caller (this container only).

Imports /root/reference/gaussctrl/gc_model.py unchanged, with sys.modules stubs for the
packages that are not installed here (nerfstudio, torchmetrics, gsplat), and runs
GaussCtrlModel.get_outputs (gc_model.py:77-241) for one data/bear camera.  The gsplat
calls are routed to the CPU-oracle emulation (tests/oracle_gsplat.py) and every argument
gc_model passes is recorded.  nerfstudio's projection_matrix is taken from the
reference's own copy, gaussctrl/ad_render.py:49-67 (projection_matrix_splatfacto),
extracted by AST so no other part of ad_render is executed.

Output: tests/golden/harness_bear_{train,eval}.npz -- inputs (Gaussian parameters,
camera), the captured gsplat call arguments, and gc_model's outputs.  The reference does
not travel to the GPU box: only these arrays do.

Run:  python tools/capture_harness.py
"""
from __future__ import annotations

import ast
import dataclasses
import json
import math
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_gsplat  # noqa: E402

CALLS = []


def _rec(name, fn):
    def wrapper(*args, **kwargs):
        CALLS.append((name, args, kwargs))
        return fn(*args, **kwargs)
    return wrapper


def _extract_function(path, name):
    src = open(path).read()
    tree = ast.parse(src)
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name == name:
            mod = ast.Module(body=[node], type_ignores=[])
            ns = {"math": math, "np": np}
            exec(compile(mod, path, "exec"), ns)
            return ns[name]
    raise KeyError(name)


def install_stubs():
    proj_np = _extract_function(os.path.join(REF, "gaussctrl/ad_render.py"),
                                "projection_matrix_splatfacto")

    def projection_matrix(znear, zfar, fovx, fovy, device="cpu"):
        # nerfstudio splatfacto.projection_matrix == ad_render.projection_matrix_splatfacto
        return torch.from_numpy(proj_np(fovx, fovy, znear, zfar)).to(device)

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Dummy:
        def __init__(self, *a, **k):
            pass

    mod("torchmetrics")
    mod("torchmetrics.image")
    mod("torchmetrics.image.lpip", LearnedPerceptualImagePatchSimilarity=_Dummy)
    mod("nerfstudio")
    mod("nerfstudio.model_components")
    mod("nerfstudio.model_components.losses", L1Loss=_Dummy, MSELoss=_Dummy,
        interlevel_loss=lambda *a, **k: None)
    mod("nerfstudio.model_components.renderers", BACKGROUND_COLOR_OVERRIDE=None)

    @dataclasses.dataclass
    class SplatfactoModelConfig:
        background_color: str = "random"
        sh_degree: int = 3
        sh_degree_interval: int = 1000

    class SplatfactoModel(torch.nn.Module):
        pass

    mod("nerfstudio.models")
    mod("nerfstudio.models.splatfacto", SplatfactoModel=SplatfactoModel,
        SplatfactoModelConfig=SplatfactoModelConfig, projection_matrix=projection_matrix)

    class Cameras:
        def __init__(self, c2w, fx, fy, cx, cy, width, height):
            self.camera_to_worlds = c2w[None]
            f = lambda v: torch.tensor([[float(v)]])
            self.fx, self.fy, self.cx, self.cy = f(fx), f(fy), f(cx), f(cy)
            self.width = torch.tensor([[int(width)]])
            self.height = torch.tensor([[int(height)]])

        @property
        def shape(self):
            return (1,)

        def rescale_output_resolution(self, s):
            assert s == 1

        def to(self, device):
            return self

    mod("nerfstudio.cameras")
    mod("nerfstudio.cameras.cameras", Cameras=Cameras)
    mod("nerfstudio.data")
    mod("nerfstudio.data.scene_box", OrientedBox=_Dummy)
    API = oracle_gsplat.API
    mod("gsplat")
    mod("gsplat.sh", num_sh_bases=lambda d: (d + 1) ** 2,
        spherical_harmonics=_rec("spherical_harmonics", API.spherical_harmonics))
    mod("gsplat.project_gaussians",
        project_gaussians=_rec("project_gaussians", API.project_gaussians))
    mod("gsplat.rasterize", rasterize_gaussians=_rec("rasterize_gaussians",
                                                     API.rasterize_gaussians))
    return Cameras


def load_gc_model():
    sys.path.insert(0, REF)
    import importlib
    return importlib.import_module("gaussctrl.gc_model")


def make_model(gc, params, step, training):
    model = gc.GaussCtrlModel.__new__(gc.GaussCtrlModel)
    torch.nn.Module.__init__(model)
    model.config = gc.GaussCtrlModelConfig()
    for k, v in params.items():
        setattr(model, k, torch.nn.Parameter(v.clone()))
    model.crop_box = None
    model.step = step
    model.device = torch.device("cpu")
    model.background_color = torch.tensor([0.1, 0.2, 0.3])
    model._get_downscale_factor = lambda: 1
    model.training = training
    return model


def main():
    Cameras = install_stubs()
    gc = load_gc_model()
    tj = json.load(open(os.path.join(REF, "data/bear/transforms.json")))
    frame = sorted(tj["frames"], key=lambda f: f["file_path"])[0]
    c2w = torch.tensor(frame["transform_matrix"], dtype=torch.float32)[:3, :4]
    # 512x512 intrinsics (transforms.json:2-7) scaled to 128x128 to keep fixtures small
    s = 128 / tj["w"]
    W = H = 128
    fx, fy, cx, cy = tj["fl_x"] * s, tj["fl_y"] * s, tj["cx"] * s, tj["cy"] * s
    cam_center = c2w[:3, 3]
    g = torch.Generator().manual_seed(42)
    n = 600
    # Gaussians around the point the camera looks at (1.5-3.5 units in front of it)
    fwd = -c2w[:3, 2]
    depth = 1.5 + 2.0 * torch.rand(n, 1, generator=g)
    lateral = (torch.rand(n, 3, generator=g) * 2 - 1) * 0.8
    params = {
        "means": cam_center + fwd * depth + lateral,
        "scales": torch.log(torch.rand(n, 3, generator=g) * 0.05 + 0.01),
        "quats": torch.randn(n, 4, generator=g),
        "opacities": torch.rand(n, 1, generator=g) * 4 - 2,
        "features_dc": torch.randn(n, 3, generator=g) * 0.5,
        "features_rest": torch.randn(n, 15, 3, generator=g) * 0.05,
    }
    out_dir = os.path.join(ROOT, "tests", "golden")
    os.makedirs(out_dir, exist_ok=True)
    for mode, step, training in (("train", 2500, True), ("eval", 0, False)):
        CALLS.clear()
        torch.manual_seed(7)  # gc_model draws torch.rand(3) for the training background
        model = make_model(gc, params, step, training)
        cam = Cameras(c2w, fx, fy, cx, cy, W, H)
        out = model.get_outputs(cam)
        rec = {}
        pname, pargs, _ = CALLS[0]
        assert pname == "project_gaussians"
        rec["proj_viewmat"] = pargs[4].detach().numpy()
        rec["proj_projmat"] = pargs[5].detach().numpy()
        rec["proj_glob_scale"] = np.float32(pargs[2])
        rec["proj_intrinsics"] = np.array(pargs[6:10], np.float64)
        rec["proj_hw"] = np.array(pargs[10:12], np.int64)
        rec["proj_tile_bounds"] = np.array(pargs[12], np.int64)
        rec["proj_scales_in"] = pargs[1].detach().numpy()
        rec["proj_quats_in"] = pargs[3].detach().numpy()
        sh = [c for c in CALLS if c[0] == "spherical_harmonics"]
        if sh:
            rec["sh_degrees_to_use"] = np.int64(sh[0][1][0])
            rec["sh_viewdirs"] = sh[0][1][1].detach().numpy()
        ras = [c for c in CALLS if c[0] == "rasterize_gaussians"]
        rec["raster_calls"] = np.int64(len(ras))
        rec["raster_background"] = ras[0][2]["background"].detach().numpy()
        rec["raster_colors_in"] = ras[0][1][5].detach().numpy()
        rec["raster_opacity_in"] = ras[0][1][6].detach().numpy()
        rec["out_rgb"] = out["rgb"].detach().numpy()
        rec["out_accumulation"] = out["accumulation"].detach().numpy()
        if out.get("depth") is not None:
            rec["out_depth"] = out["depth"].detach().numpy()
        rec["mat_view"] = out["mat_view"].detach().numpy()
        rec["mat_proj"] = out["mat_proj"].detach().numpy()
        rec.update({f"param_{k}": v.numpy() for k, v in params.items()})
        rec["c2w"] = c2w.numpy()
        rec["camera"] = np.array([fx, fy, cx, cy, W, H], np.float64)
        rec["step"] = np.int64(step)
        path = os.path.join(out_dir, f"harness_bear_{mode}.npz")
        np.savez_compressed(path, **rec)
        print(path, os.path.getsize(path), "bytes;", len(CALLS), "gsplat calls")


if __name__ == "__main__":
    main()
