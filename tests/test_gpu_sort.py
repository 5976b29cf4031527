"""The LSD radix sort (C ABI gsplat_sort_isect_pairs: reduce-then-scan passes -- digit counts,
row scans, stable LDS-ranked scatter) vs numpy's stable sort, from one tile to BASELINE-scale
intersection counts, on a poisoned workspace."""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("n,bits,hi", [
    (1, 13, 4624), (100, 13, 4624), (4096, 13, 4624), (4097, 13, 4624), (20000, 41, 1 << 41),
    (100000, 32, 1 << 32), (1000000, 32, 1 << 32), (8000000, 13, 4624),
    (300000, 16, 3),          # heavy duplicates: stability is what orders the values
    (50000, 64, 1 << 62),     # full-width 64-bit keys (8 passes)
])
def test_radix_sort_matches_stable_sort(gpu, n, bits, hi):
    rng = np.random.default_rng(n + bits)
    keys = rng.integers(0, hi, size=n, dtype=np.int64)
    vals = np.arange(n, dtype=np.int32)
    k, v = torch.from_numpy(keys).to(gpu), torch.from_numpy(vals).to(gpu)
    ko, vo = torch.empty_like(k), torch.empty_like(v)
    wsz = _lib.query("gsplat_sort_isect_pairs_workspace_size", n)
    ws = torch.full((wsz,), 0xAB, dtype=torch.uint8, device=gpu)  # poisoned workspace
    P = _lib.ptr
    _lib.call("gsplat_sort_isect_pairs", n, bits, P(k), P(v), P(ko), P(vo), P(ws), wsz,
              _lib.stream(gpu))
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(ko.cpu().numpy(), keys[order])
    np.testing.assert_array_equal(vo.cpu().numpy(), vals[order])
