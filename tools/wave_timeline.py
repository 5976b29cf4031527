"""Per-wave timeline of the raster backward (gsplat_debug_wave_log): how long waves live, when
they start, how busy each SIMD is and how long the tail is.  BWD selects the backward
geometries (gsplat_debug_set_raster_variant bwd_pxl: 1 blocks, 2 strips), CFG the bench
config."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
# the gsplat_debug_* switches live in the test library (include/gsplat_mi355x.h "test hooks")
os.environ.setdefault("GSPLAT_MI355X_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                        "..", "gaussctrl_exp_amd",
                                                        "libgsplat_mi355x_hooks.so"))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

cfg = os.environ.get("CFG", "headline")
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
N, H, W = sc.num_points, cam.height, cam.width
P, st = _lib.ptr, _lib.stream(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
tb = cam.tile_bounds
T = tb[0] * tb[1]
torch.manual_seed(0)
colors = torch.rand(N, 3, device=dev)
opac = torch.sigmoid(sc.opacities).contiguous()
bg = torch.rand(3, device=dev)
out = torch.empty(H, W, 3, device=dev); fT = torch.empty(H, W, device=dev)
fi = torch.empty(H, W, device=dev, dtype=torch.int32)
v_out = torch.randn(H, W, 3, device=dev); v_a = torch.randn(H, W, device=dev)
wsz = _lib.query("gsplat_rasterize_backward_workspace_size", N, 3)
ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
g = [torch.zeros(N, k, device=dev) for k in (2, 3, 3, 1)]
_lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
          P(conics), P(colors), P(opac), P(bg), P(out), P(fT), P(fi), st)

def fwd():
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(bg), P(out), P(fT), P(fi), st)

def bwd():
    _lib.call("gsplat_rasterize_backward", tb[0], tb[1], H, W, 3, N, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(bg), P(fT), P(fi), P(v_out), P(v_a), 0.99,
              *[P(x) for x in g], P(ws), wsz, st)

log = torch.zeros(4 * T * 5, dtype=torch.int64, device=dev)
runs = [("bwd", int(x)) for x in os.environ.get("BWD", "2,1").split(",") if x]
if os.environ.get("FWD", "1") == "1":
    runs.append(("fwd", 0))
for kind, f in runs:
    _lib.call("gsplat_debug_set_raster_variant", 1, f if kind == "bwd" else 0, 0)
    fn = bwd if kind == "bwd" else fwd
    for _ in range(3):
        fn()
    log.zero_()
    _lib.call("gsplat_debug_wave_log", P(log))
    fn()
    torch.cuda.synchronize()
    _lib.call("gsplat_debug_wave_log", None)
    L = log.view(-1, 5).cpu().numpy()
    L = L[L[:, 1] > 0]
    t0 = L[:, 0].min()
    s = (L[:, 0] - t0) / 100.0  # us
    e = (L[:, 1] - t0) / 100.0
    d = e - s
    span = e.max()
    hw, xcc = L[:, 2], L[:, 3]
    simd = (xcc << 16) | ((hw >> 4) & 0xFFF)
    us, inv = np.unique(simd, return_inverse=True)
    busy = np.bincount(inv, weights=d)
    last = np.zeros(len(us)); np.maximum.at(last, inv, e)
    nw = np.bincount(inv)
    print(f"== {cfg} {kind} geometry={f}: {len(L)} waves on {len(us)} SIMDs; span {span:.1f} us")
    print(f"  wave duration us: mean {d.mean():.1f} p50 {np.median(d):.1f} p90 "
          f"{np.percentile(d, 90):.1f} max {d.max():.1f}")
    print(f"  wave start us: p50 {np.median(s):.1f} p90 {np.percentile(s, 90):.1f} "
          f"max {s.max():.1f}; started after 20% of span: {(s > 0.2 * span).mean():.3f}")
    print(f"  ends: 50% by {np.percentile(e, 50):.1f}, 90% by {np.percentile(e, 90):.1f}, "
          f"99% by {np.percentile(e, 99):.1f}, all by {span:.1f}")
    print(f"  waves/SIMD mean {nw.mean():.2f} max {nw.max()}; SIMD last-end p10 "
          f"{np.percentile(last, 10):.1f} p50 {np.median(last):.1f}")
    bins_t = np.linspace(0, span, 11)
    act = [int(((s <= t) & (e > t)).sum()) for t in bins_t[:-1] + span / 20]
    print(f"  resident waves at 5%,15%..95% of span: {act}")
_lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)


def simulate(dur, order, slots):
    """Greedy list schedule: waves in `order` each take the earliest free slot of `slots`
    (first-order model of the dispatcher; durations held at their measured values)."""
    import heapq
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for w in order:
        t = heapq.heappop(free)
        e = t + dur[w]
        end = max(end, e)
        heapq.heappush(free, e)
    return end


# Schedule estimates from the last measured kernel of each kind (SIM=1): dispatch order as
# measured (model check), waves longest-first, and 8-tile chunks (the XCD chunk of the block
# order) longest-chunk-first with the chunk's tiles kept together.
if os.environ.get("SIM", "1") == "1":
    for kind, f in runs:
        _lib.call("gsplat_debug_set_raster_variant", 1, f if kind == "bwd" else 0, 0)
        fn = bwd if kind == "bwd" else fwd
        fn()
        log.zero_()
        _lib.call("gsplat_debug_wave_log", P(log))
        fn()
        torch.cuda.synchronize()
        _lib.call("gsplat_debug_wave_log", None)
        L = log.view(-1, 5).cpu().numpy()
        L = L[L[:, 1] > 0]
        t0 = L[:, 0].min()
        s, e = (L[:, 0] - t0) / 100.0, (L[:, 1] - t0) / 100.0
        dur = e - s
        slot = L[:, 4]
        resident = int(max(((s <= t) & (e > t)).sum() for t in np.linspace(0, e.max(), 50)))
        disp = np.argsort(s, kind="stable")
        lpt = np.argsort(-dur, kind="stable")
        chunk = slot // 8
        csum = np.bincount(chunk, weights=dur)
        corder = np.argsort(-csum[chunk], kind="stable")
        corder = corder[np.lexsort((slot[corder], -csum[chunk[corder]]))]
        print(f"== {cfg} {kind} geometry={f}: measured span {e.max():.1f} us, {resident} slots; "
              f"simulated dispatch order {simulate(dur, disp, resident):.1f}, waves longest-first "
              f"{simulate(dur, lpt, resident):.1f}, 8-tile chunks longest-first "
              f"{simulate(dur, corder, resident):.1f}; ideal sum/slots "
              f"{dur.sum() / resident:.1f}, longest wave {dur.max():.1f}")
    _lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)
