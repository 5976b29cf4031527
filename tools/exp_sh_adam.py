"""The N > 1 train step's SH-feature update at the headline / c4 sizes: the multi-view table
kernel over R dense view records (gsplat_compute_sh_backward_view_table) followed by the
multi-tensor Adam of features_dc / features_rest (gsplat_adam_step), against the table kernel
with that Adam fused in (gsplat_compute_sh_backward_view_table_adam).  Also the geometry
groups' Adam alone (11 floats per Gaussian) -- the other Adam the N > 1 step runs.
Usage: python tools/exp_sh_adam.py [N ...]   (default 1000000 2000000; R = 8)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from gaussctrl_exp_amd import _lib  # noqa: E402
from gaussctrl_exp_amd.optim import FusedAdam  # noqa: E402

dev = torch.device("cuda:0")
K, R = 16, 8


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for n in [int(x) for x in sys.argv[1:]] or [1_000_000, 2_000_000]:
    means = torch.randn(n, 3, device=dev)
    recs = [torch.randn(3 * n + 4, device=dev) for _ in range(R)]
    tab = ctypes.cast((ctypes.c_void_p * R)(*[r.data_ptr() for r in recs]), ctypes.c_void_p)
    caps = ctypes.cast((ctypes.c_longlong * R)(*([-1] * R)), ctypes.c_void_p)
    dc = torch.nn.Parameter(torch.randn(n, 3, device=dev))
    rest = torch.nn.Parameter(torch.randn(n, K - 1, 3, device=dev))
    geo = [torch.nn.Parameter(torch.randn(n, c, device=dev)) for c in (3, 3, 4, 1)]
    opt = FusedAdam([{"params": [dc], "lr": 2.5e-3, "name": "features_dc"},
                     {"params": [rest], "lr": 1.25e-4, "name": "features_rest"}], eps=1e-15)
    gopt = FusedAdam([{"params": [p], "lr": 1e-3, "name": f"g{i}"} for i, p in enumerate(geo)],
                     eps=1e-15)
    for p in geo:
        p.grad = torch.randn_like(p)
    st = _lib.stream(dev)
    v_dc = torch.empty(n, 3, device=dev)
    v_rest = torch.empty(n, K - 1, 3, device=dev)

    def unfused():
        _lib.call("gsplat_compute_sh_backward_view_table", n, 3, 3, R, _lib.ptr(means), tab, caps,
                  _lib.ptr(v_dc), _lib.ptr(v_rest), st)
        dc.grad, rest.grad = v_dc, v_rest
        opt.step()

    def table_only():
        _lib.call("gsplat_compute_sh_backward_view_table", n, 3, 3, R, _lib.ptr(means), tab, caps,
                  _lib.ptr(v_dc), _lib.ptr(v_rest), st)

    def fused():
        (pd, md, vd, lr_d), (pr, mr, vr, lr_r) = opt.next_step_groups([dc, rest])
        P = _lib.ptr
        _lib.call("gsplat_compute_sh_backward_view_table_adam", n, 3, 3, R, P(means), tab, caps,
                  P(pd), P(pr), P(md), P(vd), P(mr), P(vr), lr_d, lr_r, opt.step_count + 1,
                  opt.betas[0], opt.betas[1], opt.eps, st)
        opt.step_count += 1

    t_tab, t_unf, t_fus = timeit(table_only), timeit(unfused), timeit(fused)
    t_geo = timeit(lambda: gopt.step())
    b_unf = n * (12 + 12 * R + 192) + n * 48 * 28
    b_fus = n * (12 + 12 * R) + n * 48 * 24
    print(f"N={n} R={R}: table {t_tab:.1f} us; table + Adam(SH) {t_unf:.1f} us "
          f"({b_unf / t_unf / 1e3:.0f} GB/s); fused {t_fus:.1f} us ({b_fus / t_fus / 1e3:.0f} GB/s); "
          f"geometry Adam {t_geo:.1f} us ({n * 11 * 28 / t_geo / 1e3:.0f} GB/s)", flush=True)
