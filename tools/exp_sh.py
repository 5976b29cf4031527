"""SH forward at the headline size (1M Gaussians, degree 3), working set above the MALL.

Round-1 result: the LDS-staged kernel runs at 42.3 us (5.1 TB/s).  A variant without LDS,
each lane loading its own 192-B row with 16-byte non-temporal loads, ran at 181 us
(1.2 TB/s) and was removed; the run() helper still takes a variant id for future variants."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gaussctrl_exp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
n, K = 1_000_000, 16
# several distinct buffers so the working set exceeds the 256 MB MALL (as in a real step)
sets = [(torch.nn.functional.normalize(torch.randn(n, 3, device=dev), dim=-1),
         torch.randn(n, K, 3, device=dev), torch.empty(n, 3, device=dev)) for _ in range(3)]


def run(v, reps=60):
    f = lambda i: _lib.call("gsplat_compute_sh_forward", n, 3, 3, _lib.ptr(sets[i % 3][0]),
                            _lib.ptr(sets[i % 3][1]), _lib.ptr(sets[i % 3][2]),
                            _lib.stream(dev))
    for i in range(6):
        f(i)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(reps):
        f(i)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    print(f"variant {v}: {us:.1f} us  ({n * (24 + 12 * K) / us / 1e3:.0f} GB/s)")
    return sets[0][2].clone()


run(0)
