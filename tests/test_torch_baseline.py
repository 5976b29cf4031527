"""The pure-PyTorch CPU baseline (oracle/torch_ref.py: bin_and_sort, rasterize_tiles,
render_fwd_bwd_sampled) that bench.py times beside the GPU, checked against the C oracle so
the baseline computes the same render it is compared with (CPU only)."""
import numpy as np
import torch

import oracle as O
import torch_ref as TR
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.scene import synthetic_scene


def _setup(n=3000, W=128, H=96, seed=1):
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=0.01, scale_hi=0.06)
    cam = synthetic_camera(W, H)
    q = sc.quats / sc.quats.norm(dim=-1, keepdim=True)
    o = O.project_forward(sc.means.numpy(), torch.exp(sc.scales).numpy(), 1.0, q.numpy(),
                          cam.viewmat.numpy(), cam.projmat.numpy(), cam.fx, cam.fy, cam.cx,
                          cam.cy, H, W, cam.tile_bounds)
    return sc, cam, o


def test_torch_binning_equals_oracle(oracle_lib):
    sc, cam, o = _setup()
    xys, depths, radii = (torch.from_numpy(a) for a in o[:3])
    gids, bins = TR.bin_and_sort(xys, depths, radii, cam.tile_bounds)
    ref = O.bin_and_sort(o[0], o[1], o[2], o[4], cam.tile_bounds)
    assert gids.numel() == ref["num_intersects"] > 0
    np.testing.assert_array_equal(gids.numpy(), ref["gaussian_ids_sorted"])
    np.testing.assert_array_equal(bins.numpy(), ref["tile_bins"])


def test_torch_tile_rasterizer_matches_oracle(oracle_lib):
    sc, cam, o = _setup()
    H, W, tb = cam.height, cam.width, cam.tile_bounds
    xys, depths, radii, conics = (torch.from_numpy(a) for a in o[:4])
    gids, bins = TR.bin_and_sort(xys, depths, radii, tb)
    g = torch.Generator().manual_seed(2)
    col = torch.rand(xys.shape[0], 3, generator=g)
    op = torch.rand(xys.shape[0], generator=g)
    bg = torch.tensor([0.3, 0.2, 0.1])
    outs = TR.rasterize_tiles(xys, conics, col, op, bg, gids, bins, range(tb[0] * tb[1]), tb, H,
                              W)
    img = torch.zeros(H * W, 3)
    alpha = torch.zeros(H * W)
    for p, im, al in outs:
        img[p] = im
        alpha[p] = al
    rimg, rT, _ = O.rasterize_forward(tb, H, W, gids.numpy().astype(np.int32), bins.numpy(),
                                      o[0], o[3], col.numpy(), op.numpy(), bg.numpy())
    np.testing.assert_allclose(img.reshape(H, W, 3).numpy(), rimg, atol=2e-6)
    np.testing.assert_allclose(alpha.reshape(H, W).numpy(), 1 - rT, atol=2e-6)


def test_sampled_fwd_bwd_runs_and_gives_gradients():
    sc = synthetic_scene(2000, 3, seed=3, scale_lo=0.01, scale_hi=0.05)
    cam = synthetic_camera(96, 64)
    total, d = TR.render_fwd_bwd_sampled(sc.means, sc.scales, sc.quats, sc.opacities,
                                         sc.features_dc, sc.features_rest, cam.viewmat,
                                         cam.projmat, cam.c2w[:3, 3], cam.fx, cam.fy, cam.cx,
                                         cam.cy, cam.height, cam.width, 3, n_tiles=8)
    assert total > 0 and d["tiles"] == 8 and d["intersects"] > 0
    assert all(gr is not None and torch.isfinite(gr).all() for gr in d["grads"])
    assert d["grads"][0].abs().max() > 0
