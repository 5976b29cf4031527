"""The schema-typed torch operator layer (csrc/torch_ops.cpp, TORCH_LIBRARY(gsplat_mi355x)).

CPU: the op library loads next to the C ABI, registers every op with a ROCm-device and a Meta
kernel and no CPU kernel (no silent fallback), and the Meta kernels give the output shapes the
C ABI writes.  GPU: each op is bit-identical to the C-ABI entry point it wraps on the same
inputs, and a graph of ops traces under torch.compile (fullgraph) through the Meta kernels.
"""
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.ops import OP_NAMES, ops

M = torch.device("meta")


def _has_kernel(name, key):
    return torch._C._dispatch_has_kernel_for_dispatch_key(f"gsplat_mi355x::{name}", key)


def test_ops_registered_with_device_and_meta_kernels_only():
    O = ops()
    for name in OP_NAMES:
        assert hasattr(O, name), name
        assert _has_kernel(name, "CUDA"), name
        assert _has_kernel(name, "Meta"), name
        assert not _has_kernel(name, "CPU"), name


def test_cpu_tensors_fail_loudly():
    with pytest.raises(NotImplementedError, match="CPU"):
        ops().sh_fwd(3, 3, torch.zeros(4, 3), torch.zeros(4, 16, 3))


def test_meta_shapes():
    O = ops()
    n, H, W, C, I = 37, 48, 64, 3, 211
    f = lambda *s: torch.empty(*s, device=M)  # noqa: E731
    i = lambda *s: torch.empty(*s, device=M, dtype=torch.int32)  # noqa: E731
    out = O.project_fwd(f(n, 3), f(n, 3), 1.0, f(n, 4), f(4, 4), f(4, 4), 50.0, 50.0, 32.0,
                        24.0, H, W, 4, 3, 0.01)
    assert [tuple(t.shape) for t in out] == [(n, 2), (n,), (n,), (n, 3), (n,), (n, 6)]
    assert [t.dtype for t in out] == [torch.float32, torch.float32, torch.int32, torch.float32,
                                      torch.int32, torch.float32]
    vm, vs, vq = O.project_bwd(f(n, 3), f(n, 3), 1.0, f(n, 4), f(4, 4), f(4, 4), 50.0, 50.0,
                               32.0, 24.0, H, W, f(n, 6), i(n), f(n, 3), f(n, 2), None, f(n, 3))
    assert (vm.shape, vs.shape, vq.shape) == ((n, 3), (n, 3), (n, 4))
    assert O.sh_fwd(3, 2, f(n, 3), f(n, 16, 3)).shape == (n, 3)
    assert O.sh_bwd(3, 2, f(n, 3), f(n, 3)).shape == (n, 16, 3)
    ids, gids = O.map_intersects(f(n, 2), f(n), i(n), i(n), 4, 3, I)
    assert (ids.shape, ids.dtype, gids.shape, gids.dtype) == ((I,), torch.int64, (I,),
                                                              torch.int32)
    ko, vo = O.sort_pairs(torch.empty(I, device=M, dtype=torch.int64), i(I), 36)
    assert (ko.shape, vo.shape) == ((I,), (I,))
    assert O.tile_bins(ko, 12).shape == (12, 2)
    img, fT, fi = O.raster_fwd(4, 3, H, W, i(I), i(12, 2), f(n, 2), f(n, 3), f(n, C), f(n, 1),
                               f(C))
    assert (img.shape, fT.shape, fi.shape, fi.dtype) == ((H, W, C), (H, W), (H, W), torch.int32)
    g = O.raster_bwd(4, 3, H, W, i(I), i(12, 2), f(n, 2), f(n, 3), f(n, C), f(n, 1), f(C),
                     f(H, W), i(H, W), f(H, W, C), None, 0.999)
    assert [tuple(t.shape) for t in g] == [(n, 2), (n, 3), (n, C), (n, 1)]


# ------------------------------------------------------------------------------------- GPU
def _case(gpu, n=3000, W=100, H=75, seed=3):
    from gaussctrl_exp_amd.camera import synthetic_camera
    from gaussctrl_exp_amd.scene import synthetic_scene
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=0.02, scale_hi=0.3, extent=4.0)
    cam = synthetic_camera(W, H)
    d = dict(means=sc.means.to(gpu).contiguous(), scales=torch.exp(sc.scales).to(gpu),
             quats=(sc.quats / sc.quats.norm(dim=-1, keepdim=True)).to(gpu).contiguous(),
             viewmat=cam.viewmat.to(gpu).contiguous(), projmat=cam.projmat.to(gpu).contiguous())
    return sc, cam, d


def _cam_args(cam):
    return (float(cam.fx), float(cam.fy), float(cam.cx), float(cam.cy), cam.height, cam.width)


@pytest.mark.gpu
def test_ops_match_c_abi_bitexact(gpu):
    """Every op against a direct ctypes call of the entry point it wraps."""
    from gaussctrl_exp_amd import quirks
    P, st = _lib.ptr, _lib.stream(gpu)
    O = ops()
    sc, cam, d = _case(gpu)
    n = d["means"].shape[0]
    tbx, tby = cam.tile_bounds[0], cam.tile_bounds[1]
    fx, fy, cx, cy, H, W = _cam_args(cam)
    got = O.project_fwd(d["means"], d["scales"], 1.0, d["quats"], d["viewmat"], d["projmat"],
                        fx, fy, cx, cy, H, W, tbx, tby, 0.01)
    ref = [torch.empty_like(t) for t in got]
    xys, depths, radii, conics, nth, cov3d = ref
    _lib.call("gsplat_project_gaussians_forward", n, P(d["means"]), P(d["scales"]), 1.0,
              P(d["quats"]), P(d["viewmat"]), P(d["projmat"]), fx, fy, cx, cy, H, W, tbx, tby,
              0.01, P(cov3d), P(xys), P(depths), P(radii), P(conics), P(nth), st)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    assert int((radii > 0).sum()) > 0

    g = torch.Generator(device="cpu").manual_seed(0)
    v_xy = torch.randn(n, 2, generator=g).to(gpu)
    v_depth = torch.randn(n, generator=g).to(gpu)
    v_conic = torch.randn(n, 3, generator=g).to(gpu)
    for vd in (v_depth, None):
        got = O.project_bwd(d["means"], d["scales"], 1.0, d["quats"], d["viewmat"],
                            d["projmat"], fx, fy, cx, cy, H, W, cov3d, radii, conics, v_xy, vd,
                            v_conic)
        ref = [torch.empty_like(t) for t in got]
        _lib.call("gsplat_project_gaussians_backward", n, P(d["means"]), P(d["scales"]), 1.0,
                  P(d["quats"]), P(d["viewmat"]), P(d["projmat"]), fx, fy, cx, cy, H, W,
                  P(cov3d), P(radii), P(conics), P(v_xy), P(vd), P(v_conic), None, None,
                  P(ref[0]), P(ref[1]), P(ref[2]), st)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)

    viewdirs = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=-1).to(gpu)
    coeffs = torch.randn(n, 16, 3, generator=g).to(gpu)
    for use in (0, 2, 3):
        col = O.sh_fwd(3, use, viewdirs, coeffs)
        ref = torch.empty_like(col)
        _lib.call("gsplat_compute_sh_forward", n, 3, use, P(viewdirs), P(coeffs), P(ref), st)
        assert torch.equal(col, ref)
        vc = O.sh_bwd(3, use, viewdirs, col)
        ref = torch.empty_like(vc)
        _lib.call("gsplat_compute_sh_backward", n, 3, use, P(viewdirs), P(col), P(ref), st)
        assert torch.equal(vc, ref)

    cum = torch.cumsum(nth, 0, dtype=torch.int32)
    I = int(cum[-1].item())
    ids, gids = O.map_intersects(xys, depths, radii, cum, tbx, tby, I)
    rids = torch.zeros_like(ids)
    rg = torch.zeros_like(gids)
    _lib.call("gsplat_map_gaussian_to_intersects", n, P(xys), P(depths), P(radii), P(cum), tbx,
              tby, P(rids), P(rg), st)
    assert torch.equal(ids, rids) and torch.equal(gids, rg)
    ks, vs = O.sort_pairs(ids, gids, 64)
    order = torch.sort(ids.cpu(), stable=True).indices
    assert torch.equal(ks.cpu(), ids.cpu()[order]) and torch.equal(vs.cpu(), gids.cpu()[order])
    T = tbx * tby
    bins = O.tile_bins(ks, max(I, T))
    rb = torch.empty_like(bins)
    _lib.call("gsplat_get_tile_bin_edges", I, P(ks), P(rb), max(I, T), st)
    assert torch.equal(bins, rb)

    colors = torch.rand(n, 3, generator=g).to(gpu)
    opac = torch.rand(n, 1, generator=g).to(gpu)
    bg = torch.rand(3, generator=g).to(gpu)
    img, fT, fi = O.raster_fwd(tbx, tby, H, W, vs, bins, xys, conics, colors, opac, bg)
    r = [torch.empty_like(t) for t in (img, fT, fi)]
    _lib.call("gsplat_rasterize_forward", tbx, tby, H, W, 3, P(vs), P(bins), P(xys), P(conics),
              P(colors), P(opac), P(bg), P(r[0]), P(r[1]), P(r[2]), st)
    for a, b in zip((img, fT, fi), r):
        assert torch.equal(a, b)

    prev = _lib.set_deterministic(True)  # fixed accumulation order: bit-comparable gradients
    try:
        v_img = torch.randn(H, W, 3, generator=g).to(gpu)
        v_alpha = torch.randn(H, W, generator=g).to(gpu)
        clamp = quirks.backward_alpha_clamp()
        for va in (v_alpha, None):
            got = O.raster_bwd(tbx, tby, H, W, vs, bins, xys, conics, colors, opac, bg, fT, fi,
                               v_img, va, clamp)
            ref = [torch.empty_like(t) for t in got]
            wsz = _lib.query("gsplat_rasterize_backward_workspace_size", n, 3)
            ws = torch.empty(max(wsz, 1), device=gpu, dtype=torch.uint8)
            _lib.call("gsplat_rasterize_backward", tbx, tby, H, W, 3, n, P(vs), P(bins), P(xys),
                      P(conics), P(colors), P(opac), P(bg), P(fT), P(fi), P(v_img), P(va),
                      clamp, P(ref[0]), P(ref[1]), P(ref[2]), P(ref[3]), P(ws), wsz, st)
            for a, b in zip(got, ref):
                assert torch.equal(a, b)
            assert float(got[0].abs().sum()) > 0
    finally:
        _lib.set_deterministic(prev)


@pytest.mark.gpu
def test_ops_rejects_bad_inputs(gpu):
    O = ops()
    with pytest.raises(RuntimeError, match="float32|Float"):
        O.sh_fwd(3, 3, torch.zeros(4, 3, device=gpu, dtype=torch.float64),
                 torch.zeros(4, 16, 3, device=gpu))
    with pytest.raises(RuntimeError, match="coeffs"):
        O.sh_fwd(3, 3, torch.zeros(4, 3, device=gpu), torch.zeros(4, 9, 3, device=gpu))
    with pytest.raises(RuntimeError, match="contiguous"):
        O.sh_fwd(3, 3, torch.zeros(3, 4, device=gpu).t(), torch.zeros(4, 16, 3, device=gpu))


@pytest.mark.gpu
def test_ops_trace_under_torch_compile(gpu):
    """project -> SH -> (eager binning) -> raster as compiled graphs (fullgraph: no breaks),
    bit-identical to the eager ops."""
    O = ops()
    sc, cam, d = _case(gpu, n=2000, W=64, H=48, seed=0)
    n = d["means"].shape[0]
    tbx, tby = cam.tile_bounds[0], cam.tile_bounds[1]
    fx, fy, cx, cy, H, W = _cam_args(cam)
    g = torch.Generator(device="cpu").manual_seed(1)
    coeffs = torch.randn(n, 16, 3, generator=g).to(gpu)
    campos = torch.randn(3, generator=g).to(gpu)

    def front(means, scales, quats, viewmat, projmat, coeffs):
        xys, depths, radii, conics, nth, cov3d = O.project_fwd(
            means, scales, 1.0, quats, viewmat, projmat, fx, fy, cx, cy, H, W, tbx, tby, 0.01)
        dirs = torch.nn.functional.normalize(means - campos, dim=-1).contiguous()
        colors = torch.clamp_min(O.sh_fwd(3, 3, dirs, coeffs) + 0.5, 0.0).contiguous()
        return xys, depths, radii, conics, nth, colors

    def back(gids, bins, xys, conics, colors, opac, bg):
        img, fT, fi = O.raster_fwd(tbx, tby, H, W, gids, bins, xys, conics, colors, opac, bg)
        return img, 1.0 - fT

    args = (d["means"], d["scales"], d["quats"], d["viewmat"], d["projmat"], coeffs)
    eager = front(*args)
    comp = torch.compile(front, backend="aot_eager", fullgraph=True)(*args)
    for a, b in zip(eager, comp):
        assert torch.equal(a, b)
    xys, depths, radii, conics, nth, colors = eager
    cum = torch.cumsum(nth, 0, dtype=torch.int32)
    I = int(cum[-1].item())
    assert I > 0
    ids, gids = O.map_intersects(xys, depths, radii, cum, tbx, tby, I)
    ks, vs = O.sort_pairs(ids, gids, 64)
    bins = O.tile_bins(ks, max(I, tbx * tby))
    opac = torch.full((n, 1), 0.5, device=gpu)
    bg = torch.zeros(3, device=gpu)
    rargs = (vs, bins, xys, conics, colors, opac, bg)
    e = back(*rargs)
    c = torch.compile(back, backend="aot_eager", fullgraph=True)(*rargs)
    for a, b in zip(e, c):
        assert torch.equal(a, b)
    assert float(e[1].max()) > 0
