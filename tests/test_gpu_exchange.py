"""Data-parallel SH-gradient exchange on the MI355X.

gsplat_compute_sh_backward_views (sum over views of Y(means - campos_r) (x) v_colors_r) is
checked against the CPU oracle's restatement (oracle.sh_backward_views) and against the sum
of single-view gsplat_compute_sh_backward calls, over every SH degree, a partial
degrees_to_use, ragged N and padded view records.  Then the whole exchange runs over RCCL at
world size 1: the render's feature gradients through ShViewExchange equal the plain ones.
"""
import socket

import numpy as np
import pytest
import torch

import oracle as O
from gaussctrl_exp_amd.sh import num_sh_bases, sh_backward_views, spherical_harmonics

pytestmark = pytest.mark.gpu


def _records(n, R, pad, seed):
    g = torch.Generator().manual_seed(seed)
    means = (torch.rand(n, 3, generator=g) * 2 - 1) * 1.5
    campos = torch.randn(R, 3, generator=g) * 4
    vcol = torch.randn(R, n, 3, generator=g)
    views = torch.zeros(R, 3 * n + 3 + pad)
    views[:, :3 * n] = vcol.reshape(R, -1)
    views[:, 3 * n:3 * n + 3] = campos
    return means, campos, vcol, views


@pytest.mark.parametrize("degree,dtu", [(0, 0), (1, 1), (2, 2), (3, 3), (3, 1), (4, 4)])
@pytest.mark.parametrize("n,R,pad", [(1000, 1, 0), (1037, 3, 1), (4096, 8, 5)])
def test_sh_backward_views_vs_oracle(gpu, oracle_lib, degree, dtu, n, R, pad):
    means, campos, vcol, views = _records(n, R, pad, seed=degree * 100 + R)
    K = num_sh_bases(degree)
    got = sh_backward_views(degree, dtu, means.to(gpu), views.to(gpu)).cpu().numpy()
    ref = O.sh_backward_views(dtu, means.numpy(), views.numpy(), K)
    assert got.shape == (n, K, 3)
    # the parity bar (1e-5 abs / 1e-4 rel): a degree-4 basis near cancellation rounds ~1e-6
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
    # the split-output variant (fused training path) writes the same values into two tensors
    from gaussctrl_exp_amd.fused import sh_backward_views_split
    v_dc, v_rest = sh_backward_views_split(degree, dtu, means.to(gpu), views.to(gpu))
    np.testing.assert_array_equal(v_dc.cpu().numpy(), got[:, 0])
    np.testing.assert_array_equal(v_rest.cpu().numpy(), got[:, 1:])
    # == the sum of the single-view HIP backward on each view's (normalised) directions
    from gaussctrl_exp_amd import _lib
    acc = torch.zeros(n, K, 3, device=gpu)
    for r in range(R):
        d = (means - campos[r]).to(gpu)
        d = d / d.norm(dim=-1, keepdim=True)
        out = torch.empty(n, K, 3, device=gpu)
        vc = vcol[r].contiguous().to(gpu)  # held: a pointer to a temporary would dangle
        _lib.call("gsplat_compute_sh_backward", n, degree, dtu, _lib.ptr(d), _lib.ptr(vc),
                  _lib.ptr(out), _lib.stream(gpu))
        acc += out
    np.testing.assert_allclose(got, acc.cpu().numpy(), rtol=1e-4, atol=1e-5)
    if dtu < degree:  # bases above degrees_to_use get zero gradient
        assert not got[:, num_sh_bases(dtu):].any()


def test_sh_backward_views_garden_r8(gpu, oracle_lib):
    """BASELINE config c4's exchange at its real size: the 2M garden Gaussians, the first 8
    garden cameras as the 8 ranks' views (R = 8), SH degree 3, vs the oracle."""
    import bench
    scene, _ = bench.make_workload("c4", 0, torch.device("cpu"))
    cams = [bench.make_workload("c4", r, torch.device("cpu"))[1] for r in range(8)]
    means = scene.means.contiguous()
    n, R, K = means.shape[0], 8, 16
    g = torch.Generator().manual_seed(44)
    views = torch.zeros(R, 3 * n + 4)
    views[:, :3 * n] = torch.randn(R, 3 * n, generator=g) * 1e-3
    for r, c in enumerate(cams):
        views[r, 3 * n:3 * n + 3] = c.c2w[:3, 3]
    got = sh_backward_views(3, 3, means.to(gpu), views.to(gpu)).cpu().numpy()
    ref = O.sh_backward_views(3, means.numpy(), views.numpy(), K)
    assert got.shape == (n, K, 3) and np.abs(ref).max() > 0
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5 * 1e-3)


def test_sh_backward_views_rejects_short_stride(gpu):
    from gaussctrl_exp_amd import _lib
    means = torch.zeros(10, 3, device=gpu)
    views = torch.zeros(2, 32, device=gpu)  # needs >= 33
    out = torch.empty(10, 16, 3, device=gpu)
    with pytest.raises(RuntimeError, match="bad args"):
        _lib.call("gsplat_compute_sh_backward_views", 10, 3, 3, 2, _lib.ptr(means),
                  _lib.ptr(views), 32, _lib.ptr(out), _lib.stream(gpu))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_exchange_over_rccl_world1_matches_plain(gpu):
    """The full path through RCCL (all_gather_into_tensor on the device) at world size 1:
    SH-feature gradients via the exchange == the plain single-view backward."""
    import torch.distributed as dist
    from gaussctrl_exp_amd.camera import synthetic_camera
    from gaussctrl_exp_amd.exchange import ShViewExchange
    from gaussctrl_exp_amd.scene import render, synthetic_scene

    from gaussctrl_exp_amd import _lib
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=gpu)
    # deterministic rasterizer backward: the two renders' float-atomic summation orders would
    # otherwise differ run to run (means.grad comes only through the rasterizer's atomics)
    prev = _lib.set_deterministic(True)
    try:
        cam = synthetic_camera(256, 192).to(gpu)
        bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
        grads = []
        for use_exchange in (False, True):
            sc = synthetic_scene(20000, 3, seed=5, device=gpu).requires_grad_()
            xchg = ShViewExchange()
            if use_exchange:
                with xchg.view(sc.means, cam.c2w[..., :3, 3]):
                    out = render(sc, cam, 3, bg)
            else:
                out = render(sc, cam, 3, bg)
            (out["rgb"] * torch.linspace(0, 1, 3, device=gpu)).sum().backward()
            assert xchg.handled == use_exchange
            grads.append([sc.features_dc.grad.cpu().numpy(),
                          sc.features_rest.grad.cpu().numpy(), sc.means.grad.cpu().numpy()])
        for a, b in zip(*grads):
            assert np.abs(b).max() > 0
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    finally:
        _lib.set_deterministic(prev)
        dist.destroy_process_group()


def test_trainstep_multirank_path_over_rccl_world1(gpu):
    """TrainStep's multi-rank configuration (SH view exchange + canonical-order all-reduces,
    what bench.py runs at N > 1) driven over RCCL at world size 1 equals the single-rank
    step, and an empty view (the caller's early background return) goes through every
    collective without a hang and leaves zero gradients."""
    import torch.distributed as dist
    from gaussctrl_exp_amd.camera import gc_camera, look_at_c2w, synthetic_camera
    from gaussctrl_exp_amd.scene import synthetic_scene
    from gaussctrl_exp_amd.train import TrainStep

    from gaussctrl_exp_amd import _lib
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=gpu)
    # deterministic rasterizer backward: bit-comparable gradients between the two steps
    prev = _lib.set_deterministic(True)
    try:
        cam = synthetic_camera(256, 192).to(gpu)
        gt = torch.rand(192, 256, 3, generator=torch.Generator().manual_seed(2)).to(gpu)
        bg = torch.tensor([0.2, 0.3, 0.4], device=gpu)
        flats = []
        for ws in (1, 2):  # 2: build the multi-rank exchange objects (the group has 1 rank)
            t = TrainStep(synthetic_scene(20000, 3, seed=6, device=gpu), sh_degree=3,
                          world_size=ws, loss="splatfacto")
            t.step(cam, gt, background=bg, optimizer=False)
            flats.append(t.flat_grad().cpu().numpy())
        assert np.abs(flats[0]).max() > 0
        np.testing.assert_allclose(flats[1], flats[0], rtol=1e-5, atol=1e-6)
        # optimiser steps: the multi-rank path updates the SH-feature groups while the other
        # groups' all-reduces are in flight, then the rest (one shared step count)
        params = []
        for ws in (1, 2):
            t = TrainStep(synthetic_scene(20000, 3, seed=6, device=gpu), sh_degree=3,
                          world_size=ws, loss="splatfacto")
            for _ in range(3):
                t.step(cam, gt, background=bg, optimizer=True)
            assert t.opt.step_count == 3
            params.append([p.detach().cpu().numpy() for p in t.params])
        for a, b in zip(*params):
            np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-6)
        away = gc_camera(look_at_c2w((0.0, 0.0, 4.0), target=(0.0, 0.0, 8.0),
                                     up=(0.0, 1.0, 0.0)), 200.0, 200.0, 128.0, 96.0, 256,
                         192).to(gpu)
        t = TrainStep(synthetic_scene(20000, 3, seed=6, device=gpu), sh_degree=3,
                      world_size=2, loss="splatfacto")
        t.step(away, gt, background=bg, optimizer=True)
        assert all(p.grad is not None and not p.grad.any() for p in t.params)
    finally:
        _lib.set_deterministic(prev)
        dist.destroy_process_group()


def _sparse_inputs(n, frac, seed, gpu):
    """radii with about `frac` visible (plus whole 64-blocks culled / visible), random gradient
    records, colours with some clamp-raised (-0.0) entries."""
    g = torch.Generator().manual_seed(seed)
    vis = torch.rand(n, generator=g) < frac
    if n >= 256:
        vis[64:128] = False
        vis[128:192] = True
    radii = torch.where(vis, torch.randint(1, 9, (n,), generator=g), torch.zeros(n, dtype=torch.int64))
    recf = 16  # floats per gradient record (gsplat_grad_records_bytes / N / 4)
    rec = torch.randn(n, recf, generator=g)
    colors = torch.rand(n, 3, generator=g)
    colors[torch.rand(n, 3, generator=g) < 0.1] = -0.0
    campos = torch.randn(3, generator=g)
    return (radii.to(torch.int32), rec, colors, campos,
            [t.to(gpu) for t in (radii.to(torch.int32), rec, colors, campos)])


def _expected_sparse(radii, rec, colors, campos, cap):
    """The sparse record (exchange_layout.h) restated in numpy."""
    n = radii.shape[0]
    W = (n + 63) // 64
    vis = (radii.numpy() > 0)
    pad = np.zeros(W * 64, dtype=bool)
    pad[:n] = vis
    bits = pad.reshape(W, 64)
    words = (bits.astype(np.uint64) << np.arange(64, dtype=np.uint64)).sum(axis=1, dtype=np.uint64)
    pop = bits.sum(axis=1).astype(np.uint32)
    prefix = np.concatenate([[0], np.cumsum(pop)[:-1]]).astype(np.uint32)
    c = colors.numpy()
    passes = (c >= 0) & ~np.signbit(c)
    v = np.where(passes, rec.numpy()[:, 5:8], 0.0).astype(np.float32)
    out = np.zeros(4 + 3 * W + 3 * cap, dtype=np.float32)
    out[:3] = campos.numpy()
    out[3:4] = np.array([vis.sum()], dtype=np.uint32).view(np.float32)
    out[4:4 + 2 * W] = words.view(np.float32)
    out[4 + 2 * W:4 + 3 * W] = prefix.view(np.float32)
    vals = v[vis]
    out[4 + 3 * W:4 + 3 * W + vals.size] = vals.reshape(-1)
    return out, int(vis.sum())


@pytest.mark.parametrize("n,frac", [(1, 1.0), (63, 0.5), (1037, 0.55), (4101, 0.3),
                                    (130_000, 0.55), (70_000, 0.0), (1_500_000, 0.55),
                                    (700_000, 0.97)])
def test_sparse_record_matches_restatement(gpu, n, frac):
    """gsplat_exchange_sparse_plan + _pack_sparse write exactly the layout exchange_layout.h
    states (bitmap, prefix, count, values in index order, camera centre), and the dense pack of
    the same inputs holds the same values at the visible rows and zeros elsewhere.  (The two
    largest cases span several scan workgroups: XS_CHUNK = 4,096 words each.)"""
    from gaussctrl_exp_amd import _lib
    from gaussctrl_exp_amd.exchange import sparse_floats
    radii, rec, colors, campos, (d_radii, d_rec, d_colors, d_campos) = _sparse_inputs(n, frac, n, gpu)
    rec_bytes = d_rec.numel() * 4
    exp_full, count = _expected_sparse(radii, rec, colors, campos, n)
    for cap in sorted({count, n}):
        send = torch.full((sparse_floats(n, n),), float("nan"), device=gpu)
        st = _lib.stream(gpu)
        _lib.call("gsplat_exchange_sparse_plan", n, _lib.ptr(d_radii), _lib.ptr(send), st)
        _lib.call("gsplat_exchange_pack_sparse", n, _lib.ptr(d_rec), rec_bytes, _lib.ptr(d_radii),
                  _lib.ptr(d_colors), _lib.ptr(d_campos), _lib.ptr(send), cap, st)
        L = sparse_floats(n, cap)
        assert _lib.query("gsplat_exchange_sparse_floats", n, cap) == L
        got = send[:L].cpu().numpy()
        exp = exp_full[:L]
        head = 4 + 3 * ((n + 63) // 64) + 3 * count
        np.testing.assert_array_equal(got[:head].view(np.uint32), exp[:head].view(np.uint32))
    dense = torch.empty(3 * n + 4, device=gpu)
    _lib.call("gsplat_exchange_pack_colors", n, _lib.ptr(d_rec), rec_bytes, _lib.ptr(d_radii),
              _lib.ptr(d_colors), _lib.ptr(d_campos), _lib.ptr(dense), _lib.stream(gpu))
    dv = dense[:3 * n].view(n, 3).cpu().numpy()
    vis = radii.numpy() > 0
    W = (n + 63) // 64
    np.testing.assert_array_equal(dv[vis].reshape(-1), exp_full[4 + 3 * W:4 + 3 * W + 3 * count])
    assert not dv[~vis].any()


@pytest.mark.parametrize("degree,dtu", [(3, 3), (3, 1), (1, 1), (0, 0)])
def test_view_table_sparse_equals_dense_bitwise(gpu, degree, dtu):
    """gsplat_compute_sh_backward_view_table over sparse records, dense records and a mix gives
    the same result bit for bit (absent rows are exact zeros), within the parity bar of the
    dense multi-view kernel."""
    import ctypes
    from gaussctrl_exp_amd import _lib
    from gaussctrl_exp_amd.exchange import sparse_floats
    from gaussctrl_exp_amd.fused import sh_backward_views_split
    n, R = 50_021, 11  # two groups of 8 views in the kernel, one partial
    g = torch.Generator().manual_seed(9)
    means = ((torch.rand(n, 3, generator=g) * 2 - 1) * 1.5).to(gpu)
    dense, sparse = [], []
    st = _lib.stream(gpu)
    for r in range(R):
        radii, rec, colors, campos, (d_radii, d_rec, d_colors, d_campos) = \
            _sparse_inputs(n, 0.2 + 0.07 * r, 100 + r, gpu)
        d = torch.empty(3 * n + 4, device=gpu)
        _lib.call("gsplat_exchange_pack_colors", n, _lib.ptr(d_rec), d_rec.numel() * 4,
                  _lib.ptr(d_radii), _lib.ptr(d_colors), _lib.ptr(d_campos), _lib.ptr(d), st)
        cap = int((radii > 0).sum()) + r  # capacities above the count are allowed
        s = torch.empty(sparse_floats(n, n), device=gpu)
        _lib.call("gsplat_exchange_sparse_plan", n, _lib.ptr(d_radii), _lib.ptr(s), st)
        _lib.call("gsplat_exchange_pack_sparse", n, _lib.ptr(d_rec), d_rec.numel() * 4,
                  _lib.ptr(d_radii), _lib.ptr(d_colors), _lib.ptr(d_campos), _lib.ptr(s), cap, st)
        dense.append(d)
        sparse.append((s, cap))
    ref_dc, ref_rest = sh_backward_views_split(degree, dtu, means, torch.stack(dense))
    K = num_sh_bases(degree)
    first = None
    for mode in ("sparse", "dense", "mix"):
        ptrs, caps = [], []
        for r in range(R):
            use_sparse = mode == "sparse" or (mode == "mix" and r % 2 == 0)
            ptrs.append(sparse[r][0].data_ptr() if use_sparse else dense[r].data_ptr())
            caps.append(sparse[r][1] if use_sparse else -1)
        v_dc = torch.empty(n, 3, device=gpu)
        v_rest = torch.empty(n, K - 1, 3, device=gpu)
        _lib.call("gsplat_compute_sh_backward_view_table", n, degree, dtu, R, _lib.ptr(means),
                  ctypes.cast((ctypes.c_void_p * R)(*ptrs), ctypes.c_void_p),
                  ctypes.cast((ctypes.c_longlong * R)(*caps), ctypes.c_void_p), _lib.ptr(v_dc),
                  _lib.ptr(v_rest) if K > 1 else None, st)
        got = (v_dc.cpu().numpy(), v_rest.cpu().numpy())
        if first is None:
            first = got
        # every record mix gives the same bits (absent rows add nothing); against the dense
        # multi-view kernel (a separately compiled basis: fma contraction may differ) the
        # parity bar
        np.testing.assert_array_equal(got[0], first[0])
        np.testing.assert_array_equal(got[1], first[1])
        np.testing.assert_allclose(got[0], ref_dc.cpu().numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(got[1], ref_rest.cpu().numpy(), rtol=1e-4, atol=1e-6)
    with pytest.raises(RuntimeError, match="capacity"):
        _lib.call("gsplat_compute_sh_backward_view_table", n, degree, dtu, 1, _lib.ptr(means),
                  ctypes.cast((ctypes.c_void_p * 1)(dense[0].data_ptr()), ctypes.c_void_p),
                  ctypes.cast((ctypes.c_longlong * 1)(n + 1), ctypes.c_void_p), _lib.ptr(v_dc),
                  _lib.ptr(v_rest) if K > 1 else None, st)


@pytest.mark.parametrize("degree,dtu", [(3, 3), (3, 1), (1, 1), (0, 0)])
@pytest.mark.parametrize("n", [50_021, 4096])
def test_view_table_adam_equals_table_then_adam(gpu, degree, dtu, n):
    """gsplat_compute_sh_backward_view_table_adam (the N > 1 train step's SH-feature Adam fused
    into the multi-view table kernel) leaves features_dc / features_rest and both moments
    bit-identical to the table kernel's gradients followed by gsplat_adam_step (FusedAdam) --
    over two consecutive steps (moments non-zero), sparse and dense records mixed, ragged N
    (dword tail) and an unaligned slab start (4096 + 1 rows into a larger buffer)."""
    import ctypes
    from gaussctrl_exp_amd import _lib
    from gaussctrl_exp_amd.exchange import sparse_floats
    from gaussctrl_exp_amd.optim import FusedAdam
    R = 5
    g = torch.Generator().manual_seed(19)
    means = ((torch.rand(n, 3, generator=g) * 2 - 1) * 1.5).to(gpu)
    st = _lib.stream(gpu)
    ptrs, caps, keep = [], [], []
    for r in range(R):
        radii, rec, colors, campos, (d_radii, d_rec, d_colors, d_campos) = \
            _sparse_inputs(n, 0.3 + 0.1 * r, 200 + r, gpu)
        if r % 2:
            d = torch.empty(3 * n + 4, device=gpu)
            _lib.call("gsplat_exchange_pack_colors", n, _lib.ptr(d_rec), d_rec.numel() * 4,
                      _lib.ptr(d_radii), _lib.ptr(d_colors), _lib.ptr(d_campos), _lib.ptr(d), st)
            ptrs.append(d.data_ptr())
            caps.append(-1)
            keep.append(d)
        else:
            cap = int((radii > 0).sum())
            s = torch.empty(sparse_floats(n, n), device=gpu)
            _lib.call("gsplat_exchange_sparse_plan", n, _lib.ptr(d_radii), _lib.ptr(s), st)
            _lib.call("gsplat_exchange_pack_sparse", n, _lib.ptr(d_rec), d_rec.numel() * 4,
                      _lib.ptr(d_radii), _lib.ptr(d_colors), _lib.ptr(d_campos), _lib.ptr(s),
                      cap, st)
            ptrs.append(s.data_ptr())
            caps.append(cap)
            keep.append(s)
    K = num_sh_bases(degree)
    tab = ctypes.cast((ctypes.c_void_p * R)(*ptrs), ctypes.c_void_p)
    cap_arr = ctypes.cast((ctypes.c_longlong * R)(*caps), ctypes.c_void_p)
    # the rest slab starts one row into its storage when n is a multiple of 4 (unaligned path)
    off = 1 if n % 4 == 0 else 0
    base_dc = torch.randn(n, 3, generator=g).to(gpu)
    store = torch.randn(n + off, max(K - 1, 1), 3, generator=g).to(gpu)
    base_rest = store[off:off + n, :K - 1]

    def params():
        dc = torch.nn.Parameter(base_dc.clone())
        buf = store.clone()
        rest = torch.nn.Parameter(buf[off:off + n, :K - 1])
        return dc, rest, buf
    # reference: table kernel -> gradients -> FusedAdam.step (gsplat_adam_step)
    dc_a, rest_a, buf_a = params()
    opt_a = FusedAdam([{"params": [dc_a], "lr": 2.5e-3, "name": "features_dc"},
                       {"params": [rest_a], "lr": 1.25e-4, "name": "features_rest"}], eps=1e-15)
    dc_b, rest_b, buf_b = params()
    opt_b = FusedAdam([{"params": [dc_b], "lr": 2.5e-3, "name": "features_dc"},
                       {"params": [rest_b], "lr": 1.25e-4, "name": "features_rest"}], eps=1e-15)
    if K > 1:
        assert rest_a.is_contiguous() and (rest_a.data_ptr() % 16 != 0) == (off == 1)
    for it in range(2):
        v_dc = torch.empty(n, 3, device=gpu)
        v_rest = torch.empty(n, K - 1, 3, device=gpu)
        _lib.call("gsplat_compute_sh_backward_view_table", n, degree, dtu, R, _lib.ptr(means),
                  tab, cap_arr, _lib.ptr(v_dc), _lib.ptr(v_rest) if K > 1 else None, st)
        dc_a.grad = v_dc
        rest_a.grad = v_rest if K > 1 else None
        opt_a.step()
        (pd, md, vd, lr_d), (pr, mr, vr, lr_r) = opt_b.next_step_groups([dc_b, rest_b])
        P = _lib.ptr
        _lib.call("gsplat_compute_sh_backward_view_table_adam", n, degree, dtu, R, P(means), tab,
                  cap_arr, P(pd), P(pr) if K > 1 else None, P(md), P(vd),
                  P(mr) if K > 1 else None, P(vr) if K > 1 else None, lr_d, lr_r,
                  opt_b.step_count + 1, opt_b.betas[0], opt_b.betas[1], opt_b.eps, st)
        opt_b.step_count += 1
        torch.cuda.synchronize()
        assert torch.equal(dc_a, dc_b), it
        assert torch.equal(opt_a.state[dc_a]["exp_avg"], opt_b.state[dc_b]["exp_avg"])
        assert torch.equal(opt_a.state[dc_a]["exp_avg_sq"], opt_b.state[dc_b]["exp_avg_sq"])
        if K > 1:
            assert torch.equal(rest_a, rest_b), it
            assert torch.equal(opt_a.state[rest_a]["exp_avg"], opt_b.state[rest_b]["exp_avg"])
            assert torch.equal(opt_a.state[rest_a]["exp_avg_sq"],
                               opt_b.state[rest_b]["exp_avg_sq"])
            # the rows around the slab were not touched
            assert torch.equal(buf_b[:off], store[:off]) and torch.equal(buf_b[off + n:],
                                                                           store[off + n:])
        assert not torch.equal(dc_b, base_dc)
