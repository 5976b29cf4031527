"""Writes the real-scene inputs of configs C3 (bear) and C4 (garden) as fixtures, so the
GPU box (which has no /root/reference) can load them: each scene's transforms.json as is
(camera poses and intrinsics), and its sparse_pc.ply seed cloud as an .npz of float32 xyz
and uint8 rgb (file coordinates; the loader applies the dataparser transform).
Run here:  python tools/make_scene_fixtures.py"""
import os
import shutil
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gaussctrl_exp_amd.scene import read_ply_points  # noqa: E402

SRC = "/root/reference/data"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

for name in ("bear", "garden"):
    shutil.copyfile(os.path.join(SRC, name, "transforms.json"),
                    os.path.join(DST, f"{name}_transforms.json"))
    xyz, rgb = read_ply_points(os.path.join(SRC, name, "sparse_pc.ply"))
    np.savez_compressed(os.path.join(DST, f"{name}_sparse_pc.npz"), xyz=xyz.numpy(),
                        rgb=rgb.numpy())
    print(name, xyz.shape)
