"""The fused training step's data-parallel path with two (four) ranks on one GPU (gloo carries the
collectives here: RCCL needs one GPU per rank, and the box has one).  Each rank renders its
own view through the fused kernels; the SH-feature gradients go through the view exchange
(gsplat_compute_sh_backward_views_split on the all-gathered colour gradients) or plain
all-reduces, the rest through all-reduces.  The result must equal the sum of the two
single-view fused gradients on both ranks, and the ranks must hold identical parameters after
Adam -- the path bench.py runs at N > 1 under RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


EYES = ((0.0, 0.0, 4.0), (1.5, 0.5, 3.6), (-1.2, -0.4, 3.7), (0.4, 1.3, 3.7))


def _views(dev):
    from gaussctrl_exp_amd.camera import gc_camera, look_at_c2w
    return [gc_camera(look_at_c2w(eye, up=(0.0, 1.0, 0.0)), 220.0, 220.0, 96.0, 64.0, 192, 128)
            .to(dev) for eye in EYES]


def _scene(dev):
    from gaussctrl_exp_amd.scene import synthetic_scene
    return synthetic_scene(6000, 3, seed=12, scale_lo=0.01, scale_hi=0.05, device=dev)


def _gt(rank, dev):
    return torch.rand(128, 192, 3, generator=torch.Generator().manual_seed(rank)).to(dev)


BG = (0.3, 0.5, 0.7)


def _worker(rank, world, port, out_dir, mode, sparse="auto", per_rank=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gaussctrl_exp_amd.train import TrainStep
    bg = torch.tensor(BG, device=dev)
    t = TrainStep(_scene(dev), sh_degree=3, world_size=world, loss="l1", render_mode="fused",
                  grad_exchange=mode, sparse_exchange=sparse)
    assert not t.fuse_adam  # multi-rank: the gradients must be summed before Adam
    # rank r renders views r*per_rank ... (several per rank: one step sums them all)
    mine = list(range(rank * per_rank, (rank + 1) * per_rank))
    cams = [_views(dev)[v] for v in mine] if per_rank > 1 else _views(dev)[rank]
    gts = [_gt(v, dev) for v in mine] if per_rank > 1 else _gt(rank, dev)
    t.step(cams, gts, background=bg, optimizer=False)
    np.save(os.path.join(out_dir, f"grad{rank}.npy"), t.flat_grad().cpu().numpy())
    if mode == "sh_views":  # the four non-SH gradients went out early, from the fused backward
        assert t.sh_exchange.early_steps == 1
        kinds = t.sh_exchange.record_kinds
        assert kinds["sparse" if sparse == "on" else "dense"] == per_rank if sparse != "auto" \
            else sum(kinds.values()) == per_rank
    for _ in range(2):
        t.step(cams, gts, background=bg)
    # (the SH-feature Adam ran inside the table kernel unless GSPLAT_MI355X_FUSE_SH_ADAM=0)
    assert t.fuse_sh_adam == (os.environ.get("GSPLAT_MI355X_FUSE_SH_ADAM", "1") != "0")
    np.save(os.path.join(out_dir, f"params{rank}.npy"),
            torch.cat([p.detach().reshape(-1) for p in t.params]).cpu().numpy())
    torch.cuda.synchronize()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world,sparse,per_rank", [
    ("sh_views", 2, "auto", 1), ("sh_views", 2, "on", 1), ("sh_views", 2, "off", 1),
    ("allreduce", 2, "auto", 1), ("sh_views", 4, "auto", 1),
    ("sh_views", 2, "on", 2),  # two views per rank: records in flight across the rank's views
])
def test_fused_ranks_sum_the_view_gradients(tmp_path, mode, world, sparse, per_rank):
    from gaussctrl_exp_amd import _lib
    from parity import assert_close
    port = _free_port()
    # deterministic rasterizer backward in every process: the per-view reference below then
    # has the very raster gradients the ranks summed, and the bar needs no outlier allowance
    os.environ["GSPLAT_MI355X_DETERMINISTIC"] = "1"
    try:
        mp.spawn(_worker, args=(world, port, str(tmp_path), mode, sparse, per_rank),
                 nprocs=world, join=True)
    finally:
        os.environ.pop("GSPLAT_MI355X_DETERMINISTIC", None)
    g0 = np.load(tmp_path / "grad0.npy")
    for r in range(1, world):  # every rank holds the same summed gradients and parameters
        np.testing.assert_array_equal(np.load(tmp_path / f"grad{r}.npy"), g0)
        np.testing.assert_array_equal(np.load(tmp_path / f"params{r}.npy"),
                                      np.load(tmp_path / "params0.npy"))
    from gaussctrl_exp_amd.train import TrainStep
    dev = torch.device("cuda:0")
    ref = 0
    prev = _lib.set_deterministic(True)
    try:
        for r in range(world * per_rank):
            t = TrainStep(_scene(dev), sh_degree=3, world_size=1, loss="l1", render_mode="fused")
            t.step(_views(dev)[r], _gt(r, dev), background=torch.tensor(BG, device=dev),
                   optimizer=False)
            ref = ref + t.flat_grad().cpu().numpy()
    finally:
        _lib.set_deterministic(prev)
    assert np.abs(ref).max() > 0
    assert_close("summed view gradients", g0, ref, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("sparse,per_rank", [("on", 1), ("off", 2)])
def test_fused_sh_adam_equals_unfused(tmp_path, sparse, per_rank):
    """The N > 1 train step with the SH-feature Adam inside the multi-view table kernel
    (GSPLAT_MI355X_FUSE_SH_ADAM, default on) leaves every parameter bit-identical to the same
    steps with the table kernel's gradients and the multi-tensor Adam (deterministic raster
    backward, so both runs sum the same gradients)."""
    world = 2
    out = {}
    os.environ["GSPLAT_MI355X_DETERMINISTIC"] = "1"
    try:
        for fuse in ("1", "0"):
            d = tmp_path / f"fuse{fuse}"
            d.mkdir()
            os.environ["GSPLAT_MI355X_FUSE_SH_ADAM"] = fuse
            mp.spawn(_worker, args=(world, _free_port(), str(d), "sh_views", sparse, per_rank),
                     nprocs=world, join=True)
            out[fuse] = [np.load(d / f"params{r}.npy") for r in range(world)]
    finally:
        os.environ.pop("GSPLAT_MI355X_DETERMINISTIC", None)
        os.environ.pop("GSPLAT_MI355X_FUSE_SH_ADAM", None)
    for r in range(world):
        np.testing.assert_array_equal(out["1"][r], out["0"][r])


def _garden_worker(rank, world, port, out_dir):
    """BASELINE config c4 as stated: the 2M-Gaussian garden scene at 1080^2, rank r rendering
    garden camera r (bench.make_workload), gradients summed across the ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from gaussctrl_exp_amd.train import TrainStep
    scene, cam = bench.make_workload("c4", rank, dev)
    cam = cam.to(dev)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(rank)).to(dev)
    t = TrainStep(scene, sh_degree=3, world_size=world, loss="l1", render_mode="fused")
    t.step(cam, gt, background=torch.tensor(BG, device=dev), optimizer=False)
    np.save(os.path.join(out_dir, f"grad{rank}.npy"), t.flat_grad().cpu().numpy())
    assert t.sh_exchange.early_steps == 1
    # the garden views see ~55 % of the Gaussians: the colour gradients travel as sparse records
    assert t.sh_exchange.record_kinds == {"sparse": 1, "dense": 0}
    t.step(cam, gt, background=torch.tensor(BG, device=dev))
    np.save(os.path.join(out_dir, f"params{rank}.npy"),
            torch.cat([p.detach().reshape(-1) for p in t.params]).cpu().numpy())
    torch.cuda.synchronize()
    dist.destroy_process_group()


def test_garden_two_views_sum(tmp_path):
    """c4 (garden, 2M Gaussians @ 1080^2, 1 view per rank, summed gradients): at world size 2
    each rank's flat gradient equals the sum of the two single-view fused gradients, and both
    ranks hold identical parameters after the Adam step (deterministic rasterizer backward)."""
    from gaussctrl_exp_amd import _lib
    from parity import assert_close
    import bench
    port = _free_port()
    os.environ["GSPLAT_MI355X_DETERMINISTIC"] = "1"
    try:
        mp.spawn(_garden_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    finally:
        os.environ.pop("GSPLAT_MI355X_DETERMINISTIC", None)
    g0 = np.load(tmp_path / "grad0.npy")
    np.testing.assert_array_equal(np.load(tmp_path / "grad1.npy"), g0)
    np.testing.assert_array_equal(np.load(tmp_path / "params1.npy"),
                                  np.load(tmp_path / "params0.npy"))
    from gaussctrl_exp_amd.train import TrainStep
    dev = torch.device("cuda:0")
    ref = None
    prev = _lib.set_deterministic(True)
    try:
        for r in range(2):
            scene, cam = bench.make_workload("c4", r, dev)
            cam = cam.to(dev)
            gt = torch.rand(cam.height, cam.width, 3,
                            generator=torch.Generator().manual_seed(r)).to(dev)
            t = TrainStep(scene, sh_degree=3, world_size=1, loss="l1", render_mode="fused")
            t.step(cam, gt, background=torch.tensor(BG, device=dev), optimizer=False)
            g = t.flat_grad().cpu().numpy()
            ref = g if ref is None else ref + g
            del t, scene
    finally:
        _lib.set_deterministic(prev)
    assert np.abs(ref).max() > 0 and g0.size == ref.size == 2_000_000 * 59
    assert_close("garden summed view gradients", g0, ref, atol=1e-6, rtol=1e-4)
