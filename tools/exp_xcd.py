"""Same-process A/B of the raster kernels' block -> tile order (gsplat_debug_set_raster_variant
flags: 255 << 20 dispatch order, 1024 contiguous run per XCD, K << 20 chunks of K block
slots dealt round-robin over the 8 XCDs, 0 the shipped default): forward and backward ms, interleaved rounds, on CFGS configs.
Gradients are checked equal up to atomic summation order."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

dev = torch.device("cuda:0")
P = _lib.ptr
# variants "K:GWxGH" (K as in the flags; GW x GH: gsplat_debug_set_tile_swizzle)
chunks = [x if ":" in x else x + ":1x1"
          for x in os.environ.get("CHUNKS", "255,-1,2,4,8,16,32").split(",")]
flag = lambda k: 1024 if k < 0 else k << 20


def apply(v):
    k, sw = v.split(":")
    gw, gh = (int(t) for t in sw.split("x"))
    _lib.call("gsplat_debug_set_raster_variant", 1, 2, flag(int(k)))
    _lib.call("gsplat_debug_set_tile_swizzle", gw, gh)


def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for cfg in os.environ.get("CFGS", "headline,c4").split(","):
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    st = _lib.stream(dev)
    N, H, W = sc.num_points, cam.height, cam.width
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args())
        I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    tb = cam.tile_bounds
    g0 = torch.Generator(device=dev).manual_seed(0)
    colors = torch.rand(N, 3, device=dev, generator=g0)
    opac = torch.sigmoid(sc.opacities).contiguous()
    bg = torch.rand(3, device=dev, generator=g0)
    out = torch.empty(H, W, 3, device=dev); fT = torch.empty(H, W, device=dev)
    fi = torch.empty(H, W, device=dev, dtype=torch.int32)
    v_out = torch.randn(H, W, 3, device=dev, generator=g0)
    v_a = torch.randn(H, W, device=dev, generator=g0)
    wsz = _lib.query("gsplat_rasterize_backward_workspace_size", N, 3)
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    g = [torch.zeros(N, k, device=dev) for k in (2, 3, 3, 1)]

    def fwd():
        _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
                  P(conics), P(colors), P(opac), P(bg), P(out), P(fT), P(fi), st)

    def bwd():
        _lib.call("gsplat_rasterize_backward", tb[0], tb[1], H, W, 3, N, P(gids), P(bins),
                  P(xys), P(conics), P(colors), P(opac), P(bg), P(fT), P(fi), P(v_out), P(v_a),
                  0.99, *[P(x) for x in g], P(ws), wsz, st)

    ref_img = None
    ref_g = None
    for k in chunks:
        apply(k)
        fwd(); bwd(); torch.cuda.synchronize()
        if ref_img is None:
            ref_img, ref_g = out.clone(), [x.clone() for x in g]
        else:
            assert torch.equal(out, ref_img), f"chunk {k}: forward differs"
            for a, b in zip(g, ref_g):
                d = ((a - b).abs() / (1e-6 + b.abs().max())).max().item()
                assert d < 1e-4, f"chunk {k}: grad differs {d}"
    res = {k: ([], []) for k in chunks}
    for rnd in range(5):
        for k in chunks:
            apply(k)
            res[k][0].append(timeit(fwd))
            res[k][1].append(timeit(bwd))
    apply("0:1x1")
    print(f"{cfg}: N={N} I={I} tiles={tb[0] * tb[1]}", flush=True)
    for k in chunks:
        print(f"  order {k:>9}: fwd {np.median(res[k][0]):.4f} ms  bwd {np.median(res[k][1]):.4f} ms",
              flush=True)
