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
* a captured binning assumes no constant depth digit, so a depth-range change (the keys' top
  byte, constant before the capture, varying within a later frame) leaves replays valid;
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
    return (float(loss.detach()), out["rgb"].detach().cpu().numpy().copy(),
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
    st = sg.stats()  # (the first call: the warm-up step and the capture, then two replays)
    assert st["captures"] == 1 and st["fallbacks"] == 0 and st["replays"] == 2, st
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


def test_graph_depth_range_change_stays_valid(gpu):
    """A captured binning assumes no constant depth digit (rasterize.bin_gaussians_speculative
    with host_wait=False): a depth range that changes between replays -- here the keys' top
    byte, constant over the frames before the capture, starts to vary within the frame -- never
    invalidates a replay; the replay equals the eager step at the new geometry."""
    sc, cam, gt, bg, tr = _setup(gpu, seed=7)
    with torch.no_grad():  # depths (camera at z = 4 looking at the origin) within [3.8, 4.2]:
        sc.means[:, 2] *= 0.2  # the keys' top byte (sign + high exponent bits) is constant
    sg = StepGraph(_stepper(tr, cam, gt, bg), gpu, params=tr.params)
    _graphed(sg, tr)
    c = cam.c2w[..., :3, 3].reshape(3)
    with torch.no_grad():
        # every other Gaussian 16x closer along its ray and 16x smaller: its depth key's
        # exponent drops by 4, so the keys' top byte now varies within the frame
        sc.means[::2] = c + (sc.means[::2] - c) / 16.0
        sc.scales[::2] += float(np.log(1.0 / 16.0))
    ref = _eager(tr, cam, gt, bg)
    got = _graphed(sg, tr)
    assert sg.stats()["fallbacks"] == 0, sg.stats()
    _close(got, ref, "replay after a depth-range change")
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


def _adam_inputs(gpu, n=30000, seed=17):
    """A fused forward's outputs, a random gradient-record buffer and random Adam state."""
    from gaussctrl_exp_amd.rasterize import BLOCK_X, BLOCK_Y
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=0.004, scale_hi=0.04).to(gpu)
    cam = synthetic_camera(320, 240).to(gpu)
    P, st = _lib.ptr, _lib.stream(gpu)
    f32 = dict(device=gpu, dtype=torch.float32)
    o = dict(xys=torch.empty((n, 2), **f32), depths=torch.empty((n,), **f32),
             radii=torch.empty((n,), device=gpu, dtype=torch.int32),
             conics=torch.empty((n, 3), **f32),
             nth=torch.empty((n,), device=gpu, dtype=torch.int32),
             colors=torch.empty((n, 3), **f32), opac=torch.empty((n,), **f32))
    ws1 = torch.empty((_lib.query("gsplat_bin_count_workspace_size", n),), device=gpu,
                      dtype=torch.uint8)
    p = [t.detach().contiguous() for t in sc.params()]
    campos = cam.c2w[..., :3, 3].reshape(3).contiguous().float()
    cam_args = (P(cam.viewmat.contiguous()), P(cam.projmat.contiguous()), P(campos),
                float(cam.fx), float(cam.fy), float(cam.cx), float(cam.cy))
    _lib.call("gsplat_fused_preprocess_forward_binned", n, 16, 3, *[P(t) for t in p], *cam_args,
              cam.height, cam.width, cam.tile_bounds[0], cam.tile_bounds[1], 0.01,
              *[P(o[k]) for k in ("xys", "depths", "radii", "conics", "nth", "colors", "opac")],
              P(ws1), ws1.numel(), st)
    g = torch.Generator().manual_seed(seed)
    rec = (torch.randn(_lib.query("gsplat_grad_records_bytes", n) // 4, generator=g) *
           1e-3).to(gpu)
    m = [torch.randn(t.shape, generator=g).to(gpu) * 1e-3 for t in p]
    v = [torch.rand(t.shape, generator=g).to(gpu) * 1e-6 for t in p]
    return sc, cam, cam_args, p, o, rec, m, v


def test_adam_device_schedule_equals_host_schedule(gpu):
    """gsplat_fused_preprocess_backward_adam_sched (the table of optim.adam_schedule_table,
    indexed by the device counter) against gsplat_fused_preprocess_backward_adam (host lr /
    step) on the same record: parameters and moments bit-identical, the counter advanced; with
    the binning's count word above the capacity nothing moves and the counter stays."""
    import ctypes
    from gaussctrl_exp_amd.optim import adam_schedule_table
    sc, cam, cam_args, p, o, rec, m, v = _adam_inputs(gpu)
    tr = TrainStep(synthetic_scene(8, 3, seed=1).to(gpu), sh_degree=3, loss="l1",
                   render_mode="fused")
    n, P, st = p[0].shape[0], _lib.ptr, _lib.stream(gpu)
    betas, eps = (0.9, 0.999), 1e-15
    for c in (0, 5, 29999, 40000):
        A = [t.clone() for t in p] + [t.clone() for t in m] + [t.clone() for t in v]
        B = [t.clone() for t in A]
        def ptrs(S):
            M = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in S[6:12]])
            V = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in S[12:18]])
            return M, V
        head = lambda S: (n, 16, 3, *[P(t) for t in S[:6]], *cam_args, cam.height, cam.width,
                          P(o["radii"]), P(o["conics"]), P(o["colors"]), P(o["opac"]), P(rec))
        MA, VA = ptrs(A)
        lrs = (ctypes.c_float * 6)(*tr._lrs_of_step(min(c, 30000)))
        _lib.call("gsplat_fused_preprocess_backward_adam", *head(A),
                  ctypes.cast(MA, ctypes.c_void_p), ctypes.cast(VA, ctypes.c_void_p),
                  ctypes.cast(lrs, ctypes.c_void_p), c + 1, *betas, eps, st)
        table = torch.from_numpy(adam_schedule_table(tr._lrs_of_step, betas, 30001)).to(gpu)
        counter = torch.tensor([c], dtype=torch.int32, device=gpu)
        MB, VB = ptrs(B)
        word = torch.tensor([100], dtype=torch.int32, device=gpu)
        _lib.call("gsplat_fused_preprocess_backward_adam_sched", *head(B),
                  ctypes.cast(MB, ctypes.c_void_p), ctypes.cast(VB, ctypes.c_void_p), P(table),
                  table.shape[1], P(counter), P(word), 100, *betas, eps, st)
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(A, B)):
            assert torch.equal(a, b), (c, k)
        assert int(counter) == c + 1
        assert not torch.equal(A[0], p[0])  # (the step moved something)
        # an overflowed binning (count word above the capacity): no update, counter kept
        C = [t.clone() for t in B]
        MC, VC = ptrs(C)
        _lib.call("gsplat_fused_preprocess_backward_adam_sched", *head(C),
                  ctypes.cast(MC, ctypes.c_void_p), ctypes.cast(VC, ctypes.c_void_p), P(table),
                  table.shape[1], P(counter), P(word), 99, *betas, eps, st)
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(C, B)):
            assert torch.equal(a, b), ("skip", c, k)
        assert int(counter) == c + 1


def test_graphed_training_steps(gpu):
    """TrainStep.step(device_schedule=True) replayed by a StepGraph next to eager host-scheduled
    steps from the same start: the losses within fp32 noise of each other step by step, the
    device counter and the host step counts in step; a capacity overflow mid-way falls back to
    an eager step (its replay moved no parameter) and the counts stay consistent."""
    torch.manual_seed(0)
    sa = synthetic_scene(40000, 3, seed=23, scale_lo=0.004, scale_hi=0.04).to(gpu)
    sb = synthetic_scene(40000, 3, seed=23, scale_lo=0.004, scale_hi=0.04).to(gpu)
    cam = synthetic_camera(512, 384).to(gpu)
    gt = torch.rand(384, 512, 3, generator=torch.Generator().manual_seed(5)).to(gpu)
    bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
    ta = TrainStep(sa, sh_degree=3, loss="splatfacto", render_mode="fused")
    tb = TrainStep(sb, sh_degree=3, loss="splatfacto", render_mode="fused")
    sg = StepGraph(lambda: tb.step(cam, gt, bg, device_schedule=True), gpu,
                   after_capture=lambda: tb.advance_step_count(-1),
                   after_replay=tb.advance_step_count)
    for k in range(6):
        la = float(ta.step(cam, gt, bg).detach())
        lb = float(sg.step().detach())
        assert abs(la - lb) <= 1e-4 * abs(la), (k, la, lb)
        assert ta.step_count == tb.step_count == tb.opt.step_count == k + 1
        assert int(tb._sched["counter"]) == tb.step_count
    st = sg.stats()
    assert st["captures"] == 1 and st["fallbacks"] == 0, st
    with torch.no_grad():
        for s in (sa, sb):
            s.scales.add_(0.7)  # I past the captured capacity
    la = float(ta.step(cam, gt, bg).detach())
    lb = float(sg.step().detach())
    assert sg.stats()["fallbacks"] == 1
    assert abs(la - lb) <= 1e-3 * abs(la), (la, lb)
    assert ta.step_count == tb.step_count == 7 and int(tb._sched["counter"]) == 7
    for k in range(2):  # captured again at the new capacity
        la = float(ta.step(cam, gt, bg).detach())
        lb = float(sg.step().detach())
        assert abs(la - lb) <= 1e-3 * abs(la), (k, la, lb)
    assert sg.stats()["captures"] == 2
    assert int(tb._sched["counter"]) == tb.step_count == 9
    for a, b in zip(sa.params(), sb.params()):
        assert torch.isfinite(b).all()
    sg.close()
