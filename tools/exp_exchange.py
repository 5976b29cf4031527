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
