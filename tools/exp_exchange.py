"""Times the multi-view SH backward (exchange.ShViewExchange's kernel) against the
single-view one at the headline size: N = 1M Gaussians, degree 3, R = 1, 2, 4, 8 views."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gaussctrl_exp_amd import _lib  # noqa: E402
from gaussctrl_exp_amd.sh import sh_backward_views  # noqa: E402

dev = torch.device("cuda:0")
n, K = 1_000_000, 16
means = torch.randn(n, 3, device=dev)
dirs = torch.nn.functional.normalize(torch.randn(n, 3, device=dev), dim=-1)
vcol = torch.randn(n, 3, device=dev)
out = torch.empty(n, K, 3, device=dev)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


us = timeit(lambda: _lib.call("gsplat_compute_sh_backward", n, 3, 3, _lib.ptr(dirs),
                              _lib.ptr(vcol), _lib.ptr(out), _lib.stream(dev)))
print(f"sh_backward (1 view): {us:.1f} us  ({(n * 24 + n * 192) / us / 1e3:.0f} GB/s)")
for R in (1, 2, 4, 8):
    views = torch.randn(R, 3 * n + 4, device=dev)
    us = timeit(lambda: sh_backward_views(3, 3, means, views))
    byts = n * 12 + R * n * 12 + n * 192
    print(f"sh_backward_views R={R}: {us:.1f} us  ({byts / us / 1e3:.0f} GB/s)")

# the view-table kernel (the fused render's exchange): dense and sparse records, R = 8 / 16
# (one and two views per GPU at 8 GPUs), N = 1M (headline) and 2M at 55 % visible (c4)
import ctypes  # noqa: E402
from gaussctrl_exp_amd.exchange import sparse_floats  # noqa: E402
for n2, frac in ((1_000_000, 1.0), (2_000_000, 0.55)):
    means2 = torch.randn(n2, 3, device=dev)
    radii = (torch.rand(n2, device=dev) < frac).to(torch.int32)
    rec = torch.randn(n2, 16, device=dev)
    cols = torch.rand(n2, 3, device=dev)
    cam = torch.zeros(3, device=dev)
    cap = int(radii.sum())
    sp = torch.empty(sparse_floats(n2, n2), device=dev)
    st = _lib.stream(dev)
    us_plan = timeit(lambda: _lib.call("gsplat_exchange_sparse_plan", n2, _lib.ptr(radii),
                                       _lib.ptr(sp), st))
    us_pack = timeit(lambda: _lib.call("gsplat_exchange_pack_sparse", n2, _lib.ptr(rec),
                                       rec.numel() * 4, _lib.ptr(radii), _lib.ptr(cols),
                                       _lib.ptr(cam), _lib.ptr(sp), cap, st))
    dn = torch.empty(3 * n2 + 4, device=dev)
    us_dense = timeit(lambda: _lib.call("gsplat_exchange_pack_colors", n2, _lib.ptr(rec),
                                        rec.numel() * 4, _lib.ptr(radii), _lib.ptr(cols),
                                        _lib.ptr(cam), _lib.ptr(dn), st))
    print(f"N={n2} visible {frac:.2f}: sparse plan {us_plan:.1f} us, pack {us_pack:.1f} us; "
          f"dense pack {us_dense:.1f} us; record {sparse_floats(n2, cap) * 4 / 1e6:.1f} MB "
          f"(dense {(3 * n2 + 4) * 4 / 1e6:.1f} MB)")
    v_dc = torch.empty(n2, 3, device=dev)
    v_rest = torch.empty(n2, 15, 3, device=dev)
    for R in (8, 16):
        for kind in ("dense", "sparse"):
            buf = dn if kind == "dense" else sp
            ptrs = (ctypes.c_void_p * R)(*([buf.data_ptr()] * R))
            caps = (ctypes.c_longlong * R)(*([-1 if kind == "dense" else cap] * R))
            us = timeit(lambda: _lib.call("gsplat_compute_sh_backward_view_table", n2, 3, 3, R,
                                          _lib.ptr(means2), ctypes.cast(ptrs, ctypes.c_void_p),
                                          ctypes.cast(caps, ctypes.c_void_p), _lib.ptr(v_dc),
                                          _lib.ptr(v_rest), st))
            print(f"  view table R={R} {kind}: {us:.1f} us")
