"""The fused step replayed as a HIP graph (graphs.StepGraph) against the same step issued
eagerly:

* fwd+bwd with the fused L1 loss: loss and image bit-identical to the eager step, the six
  gradients within the parity bar (the raster backward's float atomics make the eager step
  itself vary at that level), over several replays;
* replays read the inputs they were captured with: an in-place parameter update is seen by
  the next replay (compared with an eager step at the new values);
* a capacity overflow (Gaussians grown in place so I exceeds the captured capacity): the
  replay reports invalid, the step is re-run eagerly (re-binning) and equals a plain eager
  step, and the next step captures again at the new capacity;
* a depth-range change that breaks a depth-sort digit the capture assumed constant: the
  same fallback;
* the no-grad forward (c2's render) bit-identical to the eager render.
"""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.graphs import StepGraph
from gaussctrl_exp_amd.scene import synthetic_scene
from gaussctrl_exp_amd.train import TrainStep

pytestmark = pytest.mark.gpu


def _setup(gpu, n=40000, W=512, H=384, seed=3):
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=0.004, scale_hi=0.04).to(gpu)
    cam = synthetic_camera(W, H).to(gpu)
    gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(seed + 1)).to(gpu)
    bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
    tr = TrainStep(sc, sh_degree=3, loss="l1", render_mode="fused")
    return sc, cam, gt, bg, tr


def _eager(tr, cam, gt, bg):
    tr.zero_grad()
    loss, out = tr.forward_backward(cam, gt, bg)
    torch.cuda.synchronize()
    return (float(loss), out["rgb"].detach().cpu().numpy().copy(),
            [p.grad.detach().cpu().numpy().astype(np.float64) for p in tr.params])


def _graphed(sg, tr):
    loss, out = sg.step()
    torch.cuda.synchronize()
    return (float(loss), out["rgb"].detach().cpu().numpy().copy(),
            [p.grad.detach().cpu().numpy().astype(np.float64) for p in tr.params])


def _close(got, ref, what):
    assert got[0] == ref[0], (what, "loss", got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1], err_msg=f"{what}: image")
    for name, a, b in zip(("means", "scales", "quats", "opacities", "dc", "rest"), got[2], ref[2]):
        scale = np.abs(b).max()
        d = np.abs(a - b)
        assert (d <= 1e-5 * scale + 1e-4 * np.abs(b)).all(), (what, name, float(d.max()), scale)


def _stepper(tr, cam, gt, bg):
    def fn():
        tr.zero_grad()
        return tr.forward_backward(cam, gt, bg)
    return fn


def test_graphed_step_equals_eager(gpu):
    sc, cam, gt, bg, tr = _setup(gpu)
    ref = _eager(tr, cam, gt, bg)
    sg = StepGraph(_stepper(tr, cam, gt, bg), gpu, params=tr.params)
    for k in range(3):
        _close(_graphed(sg, tr), ref, f"replay {k}")
    st = sg.stats()
    assert st["captures"] == 1 and st["fallbacks"] == 0 and st["replays"] == 3, st
    # an in-place parameter update is seen by the next replay
    with torch.no_grad():
        sc.opacities.add_(0.25)
        sc.means.add_(0.002)
    got = _graphed(sg, tr)
    ref2 = _eager(tr, cam, gt, bg)
    _close(got, ref2, "after update")
    assert sg.stats()["fallbacks"] == 0
    sg.close()


def test_graph_capacity_overflow_falls_back(gpu):
    sc, cam, gt, bg, tr = _setup(gpu, seed=5)
    sg = StepGraph(_stepper(tr, cam, gt, bg), gpu, params=tr.params)
    _graphed(sg, tr)
    cap = sg.specs[0].cap
    with torch.no_grad():
        sc.scales.add_(0.7)  # ~2x larger footprints: I well past the captured capacity
    ref = _eager(tr, cam, gt, bg)
    got = _graphed(sg, tr)  # replay invalid -> the eager re-run
    st = sg.stats()
    assert st["fallbacks"] == 1, st
    assert sg.graph is None
    _close(got, ref, "fallback")
    got2 = _graphed(sg, tr)  # captured again, at the grown capacity
    st = sg.stats()
    assert st["captures"] == 2 and st["fallbacks"] == 1, st
    assert sg.specs[0].cap > cap
    _close(got2, ref, "recaptured")
    sg.close()


def test_graph_depth_range_violation_falls_back(gpu):
    sc, cam, gt, bg, tr = _setup(gpu, seed=7)
    sg = StepGraph(_stepper(tr, cam, gt, bg), gpu, params=tr.params)
    _graphed(sg, tr)
    c = cam.c2w[..., :3, 3].reshape(3)
    with torch.no_grad():  # every Gaussian 16x closer along its ray, 16x smaller: about the
        # same image, but each depth key's exponent moves by 4 (its top byte changes)
        sc.means.copy_(c + (sc.means - c) / 16.0)
        sc.scales.add_(float(np.log(1.0 / 16.0)))
    ref = _eager(tr, cam, gt, bg)
    got = _graphed(sg, tr)
    assert sg.stats()["fallbacks"] == 1, sg.stats()
    _close(got, ref, "violation fallback")
    _close(_graphed(sg, tr), ref, "recaptured")
    sg.close()


def test_graphed_forward_only_equals_eager(gpu):
    sc = synthetic_scene(100000, 0, seed=13, scale_lo=0.004, scale_hi=0.05).to(gpu)
    cam = synthetic_camera(512, 512).to(gpu)
    bg = torch.zeros(3, device=gpu)

    def fn():
        with torch.no_grad():
            return render_fused(sc, cam, 0, bg)
    ref = fn()["rgb"].cpu().numpy()
    sg = StepGraph(fn, gpu)
    for _ in range(3):
        got = sg.step()["rgb"]
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), ref)
    assert sg.stats()["captures"] == 1 and sg.stats()["fallbacks"] == 0
    sg.close()
